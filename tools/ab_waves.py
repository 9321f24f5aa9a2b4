"""A/B of k_verify_halved register bounds (2 vs 3 waves/SIMD) in ONE process,
interleaved rounds (cdna_hip_programming.md 5.4 rule 24)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xrpl-coa-prototype_amd"))
import torch  # noqa: E402

import coa_crypto  # noqa: E402
import workloads  # noqa: E402


def main():
    coa_crypto.init(1)
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(dev)
    torch.cuda.set_stream(st)
    res = {}
    for n in (65536, 524288):
        seeds = torch.from_numpy(workloads.key_seeds(n)).to(dev)
        msgs = torch.from_numpy(workloads.messages(n)).to(dev)
        pks = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        sigs = torch.empty((n, 64), dtype=torch.uint8, device=dev)
        coa_crypto.sign_many_device(0, seeds, msgs, pks, sigs, st)
        k = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        out = torch.ones(n, dtype=torch.uint8, device=dev)
        ws = torch.empty(coa_crypto.verify_workspace_bytes(n), dtype=torch.uint8, device=dev)
        coa_crypto.challenge_many_device(0, msgs, pks, sigs, k, st)
        for rnd in range(4):
            for w in ("2", "3"):
                os.environ["COA_VERIFY_WAVES"] = w
                coa_crypto.verify_prehashed_many_device(0, k, pks, sigs, out, ws, st)
                torch.cuda.synchronize()
                assert int(out.sum()) == 0
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(5):
                    coa_crypto.verify_prehashed_many_device(0, k, pks, sigs, out, ws, st)
                e1.record(st)
                torch.cuda.synchronize()
                res.setdefault((n, w), []).append(e0.elapsed_time(e1) / 5)
    for (n, w), v in sorted(res.items()):
        print(f"n={n:7d} waves={w}: median {sorted(v)[len(v)//2]:.3f} ms  min {min(v):.3f}  -> {n / (min(v) * 1e-3) / 1e6:.1f} M verify/s")


if __name__ == "__main__":
    main()
