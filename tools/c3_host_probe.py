"""Probe: the host-pointer C3 round (10,000 certificates, committee 100, one
coa_certificate_verify_many call per round from C, tools/latc.c) under the
pipelined certificate path's switches, read per call: COA_CERT_BUFFERS
(chunks in flight) x COA_CERT_CHUNK_JOBS x COA_CERT_RAMP (smaller first
chunks); C3_PROBE_CONFIGS="bufs:chunk:ramp,..." replaces the default list.  COA_PACK_THREADS is read once per
process (CopyPool), so it is set by the caller.  One JSON line per
configuration, plus the pipeline's own pack / wait split (COA_CERT_TRACE) on
stderr for one call each.

usage: python tools/c3_host_probe.py [calls]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xrpl-coa-prototype_amd"))
sys.path.insert(0, ROOT)

CONFIGS = [(2, 1 << 17, 0), (3, 1 << 17, 0), (4, 1 << 17, 0), (3, 1 << 16, 0), (4, 1 << 16, 0), (4, 1 << 15, 0)]
if os.environ.get("C3_PROBE_CONFIGS"):
    CONFIGS = [tuple(int(x) for x in c.split(":")) for c in os.environ["C3_PROBE_CONFIGS"].split(",")]


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    import numpy as np
    import torch  # noqa: F401  (one HIP runtime: torch's)

    import bench
    import certificates as C
    import coa_crypto

    coa_crypto.init(0)
    lib = bench._latc()
    vp, sz, ci, dp = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_double)
    lib.latc_certificates_many.argtypes = [vp] * 9 + [sz, vp, ci, ci, dp]
    lib.latc_certificates_many.restype = ci
    n_certs = 10000
    committee, batch = C.synth_certificates(n_certs, committee_size=100, n_payload=32, seed=3)
    committee.register()
    hd = np.frombuffer(b"".join(batch.header_inputs) + bytes(16), np.uint8)
    hoff = np.zeros(n_certs + 1, np.uint64)
    hoff[1:] = np.cumsum([len(h) for h in batch.header_inputs])
    arrs = [hd, hoff, np.ascontiguousarray(batch.ids), np.ascontiguousarray(batch.authors),
            np.ascontiguousarray(batch.header_sigs), np.full(n_certs, batch.round, np.uint64),
            np.ascontiguousarray(batch.vote_pks), np.ascontiguousarray(batch.vote_sigs),
            np.ascontiguousarray(batch.offsets)]
    ptrs = [a.ctypes.data for a in arrs]
    expect = np.zeros(n_certs, np.uint8)
    el = ctypes.c_double()
    for bufs, chunk, ramp in CONFIGS:
        os.environ["COA_CERT_BUFFERS"] = str(bufs)
        os.environ["COA_CERT_CHUNK_JOBS"] = str(chunk)
        os.environ["COA_CERT_RAMP"] = str(ramp)
        assert lib.latc_certificates_many(*ptrs, n_certs, expect.ctypes.data, 2, 1, ctypes.byref(el)) == 0
        os.environ["COA_CERT_TRACE"] = "1"
        assert lib.latc_certificates_many(*ptrs, n_certs, expect.ctypes.data, 1, 1, ctypes.byref(el)) == 0
        del os.environ["COA_CERT_TRACE"]
        best = None
        for _ in range(3):
            assert lib.latc_certificates_many(*ptrs, n_certs, expect.ctypes.data, calls, 1, ctypes.byref(el)) == 0
            best = el.value if best is None else min(best, el.value)
        print(json.dumps({"pack_threads": os.environ.get("COA_PACK_THREADS", "8"), "buffers": bufs,
                          "chunk_jobs": chunk, "ramp": ramp, "certs_per_s": round(n_certs * calls / best, 1),
                          "ms_per_round": round(best / calls * 1e3, 3)}), flush=True)


if __name__ == "__main__":
    main()
