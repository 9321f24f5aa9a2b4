"""Probe: single-certificate kernel time of the fused latency path, split by
role -- full C3 header (27 SHA-512 blocks) vs a one-block header (signature
path only) vs zero votes (header path only); HIP events on one stream."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xrpl-coa-prototype_amd"))

import numpy as np  # noqa: E402


def main():
    import torch

    import certificates as C
    import coa_crypto

    os.environ["COA_CERT_LANES"] = sys.argv[1] if len(sys.argv) > 1 else "64"
    coa_crypto.init(1)
    committee, batch = C.synth_certificates(4, committee_size=100, n_payload=32, seed=3)
    committee.register()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a).copy()).to(dev)  # noqa: E731

    def run(hdr, nvotes, label):
        hoff = np.array([0, len(hdr)], np.int64)
        voff = np.array([0, nvotes], np.int64)
        d = [T(np.frombuffer(hdr, np.uint8)) if hdr else T(np.zeros(16, np.uint8)), T(hoff), T(batch.ids[:1]),
             T(batch.authors[:1]), T(batch.header_sigs[:1]), T(np.array([batch.round], np.int64)),
             T(batch.vote_pks[:max(nvotes, 1)]), T(batch.vote_sigs[:max(nvotes, 1)]), T(voff)]
        st = torch.zeros(1, dtype=torch.int32, device=dev)
        for _ in range(3):
            coa_crypto.certificate_verify_many_device(0, *d, st, stream)
        torch.cuda.synchronize()
        ts = []
        for _ in range(30):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            coa_crypto.certificate_verify_many_device(0, *d, st, stream)
            e1.record(stream)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        print(json.dumps({"case": label, "status": int(st.item()), "us_min": round(min(ts), 1),
                          "us_p50": round(float(np.median(ts)), 1)}), flush=True)

    full = batch.header_inputs[0]
    run(full, 67, "full C3 certificate (27-block header, 1 + 67 signatures)")
    run(full[:100], 67, "1-block header, 1 + 67 signatures")
    run(full, 0, "27-block header, header signature only")
    run(full[:100], 0, "1-block header, header signature only")
    run(full[:100], 3, "1-block header, 1 + 3 signatures")
    # the header chain's cost per block: both of these are header-bound
    run(full + full, 0, "54-block header, header signature only (slope vs 27)")
    run(full + full + full + full, 0, "107-block header, header signature only")


if __name__ == "__main__":
    main()
