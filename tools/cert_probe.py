"""Probe: Certificate::verify latency / throughput of the fused path (f2+f3)
vs the stepwise path, committee 100 (C3 shape).  Prints JSON lines."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xrpl-coa-prototype_amd"))

import numpy as np  # noqa: E402


def main():
    import torch

    import certificates as C
    import coa_crypto

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    coa_crypto.init(1)
    committee, batch = C.synth_certificates(n, committee_size=100, n_payload=32, seed=3)
    t0 = time.perf_counter()
    committee.register()
    reg_ms = (time.perf_counter() - t0) * 1e3
    print(json.dumps({"register_ms": round(reg_ms, 2)}), flush=True)
    # latency: one certificate, host pointers, prepared arrays
    for lanes in ("64", "1"):
        os.environ["COA_CERT_LANES"] = lanes
        lat = []
        for i in range(300):
            c = i % n
            lo, hi = int(batch.offsets[c]), int(batch.offsets[c + 1])
            args = (batch.header_inputs[c], bytes(batch.ids[c]), bytes(batch.authors[c]), bytes(batch.header_sigs[c]),
                    batch.round, batch.vote_pks[lo:hi], batch.vote_sigs[lo:hi])
            t1 = time.perf_counter()
            st = coa_crypto.certificate_verify(*args, rng_seed=1)
            lat.append(time.perf_counter() - t1)
            assert st == 0
        lat = np.array(lat[20:]) * 1e3
        print(json.dumps({"lanes": lanes, "p50_ms": round(float(np.percentile(lat, 50)), 4),
                          "p99_ms": round(float(np.percentile(lat, 99)), 4)}), flush=True)
    del os.environ["COA_CERT_LANES"]
    # throughput, host pointers
    for lanes in ("1", "64"):
        os.environ["COA_CERT_LANES"] = lanes
        v = C.verify_certificate_batch(batch, committee)
        assert int(v.sum()) == 0
        rounds = np.full(n, batch.round, np.uint64)
        t1 = time.perf_counter()
        st = coa_crypto.certificate_verify_many(batch.header_inputs, batch.ids, batch.authors, batch.header_sigs,
                                                rounds, batch.vote_pks, batch.vote_sigs, batch.offsets)
        el = time.perf_counter() - t1
        assert int(st.sum()) == 0
        print(json.dumps({"lanes": lanes, "host_many_certs_per_s": round(n / el, 1), "ms": round(el * 1e3, 2)}),
              flush=True)
    # throughput, device-resident
    dev = torch.device("cuda", 0)
    hdata = torch.from_numpy(np.frombuffer(b"".join(batch.header_inputs), np.uint8).copy()).to(dev)
    hoff = np.zeros(n + 1, np.uint64)
    hoff[1:] = np.cumsum([len(h) for h in batch.header_inputs])
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    d_hoff = T(hoff.view(np.int64))
    d_ids, d_or, d_hs = T(batch.ids), T(batch.authors), T(batch.header_sigs)
    d_rounds = T(np.full(n, batch.round, np.int64))
    d_vp, d_vs = T(batch.vote_pks), T(batch.vote_sigs)
    d_voff = T(batch.offsets.view(np.int64))
    status = torch.empty(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream(dev)
    for lanes in ("1", "64"):
        os.environ["COA_CERT_LANES"] = lanes
        for _ in range(2):
            coa_crypto.certificate_verify_many_device(0, hdata, d_hoff, d_ids, d_or, d_hs, d_rounds, d_vp, d_vs,
                                                      d_voff, status, stream)
        torch.cuda.synchronize()
        assert int(status.abs().sum().item()) == 0, status.unique()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(5):
            coa_crypto.certificate_verify_many_device(0, hdata, d_hoff, d_ids, d_or, d_hs, d_rounds, d_vp, d_vs,
                                                      d_voff, status, stream)
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        print(json.dumps({"lanes": lanes, "device_certs_per_s": round(n / (ms * 1e-3), 1), "ms": round(ms, 3),
                          "votes_per_s": round(int(batch.offsets[-1]) / (ms * 1e-3), 1)}), flush=True)
    # stepwise host path for reference
    t1 = time.perf_counter()
    v = C.verify_certificate_batch_stepwise(batch, committee)
    el = time.perf_counter() - t1
    print(json.dumps({"stepwise_certs_per_s": round(n / el, 1)}), flush=True)


if __name__ == "__main__":
    main()
