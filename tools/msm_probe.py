"""Time the Pippenger verify_batch path (coa_ed25519_verify_batch_device) on
HBM-resident inputs at several batch sizes, beside the per-signature
verify_strict device path on the same triples.

usage: python tools/msm_probe.py [n ...]     (default 65536 2097152)
Prints one JSON line per size.  COA_MSM_RUN selects the bucket run length."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xrpl-coa-prototype_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import coa_crypto  # noqa: E402
from workloads import key_seeds, messages  # noqa: E402


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [65536, 2097152]
    coa_crypto.init(1)
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(0)  # explicit: a NULL handle would mean the engine's own stream
    for n in sizes:
        m = torch.from_numpy(np.tile(messages(1), (n, 1))).to(dev)
        seeds = torch.from_numpy(key_seeds(n)).to(dev)
        pk = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        sg = torch.empty((n, 64), dtype=torch.uint8, device=dev)
        coa_crypto.sign_many_device(0, seeds, m, pk, sg, stream=st)
        st.synchronize()
        msg = m[0].contiguous()
        out = torch.ones(1, dtype=torch.uint8, device=dev)
        ws = torch.empty(coa_crypto.verify_batch_workspace_bytes(n), dtype=torch.uint8, device=dev)
        for _ in range(2):
            coa_crypto.verify_batch_device(0, msg, pk, sg, out, rng_seed=5, workspace=ws, stream=st)
        torch.cuda.synchronize()
        reps = 10 if n <= 262144 else 4
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            coa_crypto.verify_batch_device(0, msg, pk, sg, out, rng_seed=5, workspace=ws, stream=st)
        e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        ok = int(out[0]) == 0
        # per-signature path on the same triples
        vout = torch.ones(n, dtype=torch.uint8, device=dev)
        vws = torch.empty(coa_crypto.verify_workspace_bytes(n), dtype=torch.uint8, device=dev)
        coa_crypto.verify_strict_many_device(0, m, pk, sg, vout, workspace=vws, stream=st)
        torch.cuda.synchronize()
        e0.record(st)
        for _ in range(reps):
            coa_crypto.verify_strict_many_device(0, m, pk, sg, vout, workspace=vws, stream=st)
        e1.record(st)
        torch.cuda.synchronize()
        vms = e0.elapsed_time(e1) / reps
        print(json.dumps({"n": n, "msm_ms": round(ms, 4), "msm_verif_per_s": round(n / ms * 1e3, 1), "msm_ok": ok,
                          "strict_ms": round(vms, 4), "strict_verif_per_s": round(n / vms * 1e3, 1),
                          "strict_ok": int(vout.sum()) == 0, "run": os.environ.get("COA_MSM_RUN", "auto")}),
              flush=True)
        del ws, vws
        time.sleep(0.1)


if __name__ == "__main__":
    main()
