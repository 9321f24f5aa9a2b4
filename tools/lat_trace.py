"""Phase timestamps (clock64) of the certificate latency kernel's first
signature job, from a build with -DCOA_LAT_TRACE.

  python tools/lat_trace.py build     (CPU: writes build/lat_trace/libcoa_verify.so)
  python tools/lat_trace.py run       (GPU: one C1-sized certificate, prints per-wave marks)

Marks: wave 0: 0 start, 1 hash done, 2 comb term loaded, 3 butterfly done,
4 P's half of the compare published; wave 2: 0 start, 1 (no hash), 2 comb
term loaded, 3 butterfly done; wave 1: 0 start, 1 power chain done, 2 compare
done (after waiting for wave 0), 5 verdict."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "xrpl-coa-prototype_amd")
OUT = os.path.join(ROOT, "build", "lat_trace")


def build():
    sys.path.insert(0, PKG)
    import build as b

    b.build()
    os.makedirs(OUT, exist_ok=True)
    obj = os.path.join(OUT, "coa_committee.o")
    subprocess.run([b.HIPCC] + b.COMMON + ["-DCOA_LAT_TRACE", "-c", os.path.join(b.CSRC, "coa_committee.hip"), "-o", obj],
                   check=True)
    objs = [obj if s == "coa_committee.hip" else os.path.join(b.OBJDIR, s + ".o") for s in b.SOURCES]
    subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o", os.path.join(OUT, "libcoa_verify.so")]
                   + objs, check=True)


def run():
    os.environ["COA_VERIFY_LIB"] = os.path.join(OUT, "libcoa_verify.so")
    sys.path.insert(0, PKG)
    import ctypes

    import numpy as np
    import torch  # noqa: F401

    import certificates as C
    import coa_crypto

    coa_crypto.init(1)
    committee, batch = C.synth_certificates(2, committee_size=4, n_payload=1, seed=3)
    committee.register()
    rounds = np.full(2, batch.round, np.uint64)
    L = coa_crypto.lib()
    f = L.coa_lat_trace
    f.argtypes = [ctypes.c_void_p]
    for rep in range(5):
        coa_crypto.certificate_verify(batch.header_inputs[0], batch.ids[0], batch.authors[0], batch.header_sigs[0],
                                      int(rounds[0]), batch.vote_pks[:3], batch.vote_sigs[:3])
        buf = (ctypes.c_ulonglong * 24)()
        f(ctypes.addressof(buf))
        t = np.array(list(buf), np.int64).reshape(3, 8)
        t0 = t[:, 0].min()
        print(json.dumps({"rep": rep, "wave0": (t[0, :6] - t0).tolist(), "wave1": (t[1, :5] - t0).tolist(),
                          "wave2": (t[2, :5] - t0).tolist()}), flush=True)


def hdr():
    """One committee-100 C3 certificate (27-block header, 67 votes) at a time:
    the header-digest block's phases and the kernel's end, microseconds from
    that block's start (GPU real-time clock, 100 MHz)."""
    os.environ["COA_VERIFY_LIB"] = os.path.join(OUT, "libcoa_verify.so")
    sys.path.insert(0, PKG)
    import ctypes

    import numpy as np
    import torch  # noqa: F401

    import certificates as C
    import coa_crypto

    coa_crypto.init(1)
    committee, batch = C.synth_certificates(2, committee_size=100, n_payload=32, seed=3)
    committee.register()
    L = coa_crypto.lib()
    f = L.coa_lat_trace_hdr
    f.argtypes = [ctypes.c_void_p]
    lo, hi = int(batch.offsets[0]), int(batch.offsets[1])
    names = ["hdr_start", "expanded", "rounds_done", "compared", "offsets_loaded", "sig0_verdict", "last_publish",
             "sig0_start", "block_loaded", "thread0_expanded", "-", "-"]
    for rep in range(6):
        coa_crypto.certificate_verify(batch.header_inputs[0], batch.ids[0], batch.authors[0], batch.header_sigs[0],
                                      int(batch.round), batch.vote_pks[lo:hi], batch.vote_sigs[lo:hi])
        buf = (ctypes.c_ulonglong * 12)()
        f(ctypes.addressof(buf))
        t = np.array(list(buf), np.int64)
        print(json.dumps({"rep": rep, **{n: round((int(t[i]) - int(t[0])) * 0.01, 2) for i, n in enumerate(names)
                                         if n != "-"}}), flush=True)


if __name__ == "__main__":
    {"build": build, "run": run, "hdr": hdr}[sys.argv[1]]()
