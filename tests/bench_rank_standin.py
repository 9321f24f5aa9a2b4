"""One rank of `bench.py --gpus N`, with the CPU oracle standing in for the
rank's GPU (test infrastructure: tests/test_bench_line.py launches it through
bench.main's own spawn path, bench.spawn_ranks / bench.rank_env).

It runs what a bench rank runs around the verify call -- the rank's
contiguous index range (sharding.rank_slice), bench.timed_steps (gloo
barrier, MAX over ranks), bench.gather_ranks and bench.headline -- and rank 0
prints the line.  The step verifies the rank's triples with the C oracle
(oracle/coa_oracle.c), the checker, never the measured path."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "xrpl-coa-prototype_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def main():
    import numpy as np
    import torch.distributed as dist

    import bench
    import coa_oracle as co
    import ed25519_ref as o
    import sharding
    import workloads

    args = bench.parse(sys.argv[1:])
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    local = int(os.environ["LOCAL_RANK"])
    dist.init_process_group("gloo")
    try:
        n = args.n
        lo, hi = sharding.rank_slice(rank, world, n)
        seeds, msgs = workloads.key_seeds(n, start=lo), workloads.messages(n, start=lo)
        pks = np.frombuffer(b"".join(o.public_key(bytes(s)) for s in seeds), np.uint8).reshape(-1, 32).copy()
        sigs = np.frombuffer(b"".join(o.sign(bytes(s), bytes(m)) for s, m in zip(seeds, msgs)),
                             np.uint8).reshape(-1, 64).copy()
        ok = [True]

        def step(i):
            ok[0] &= int(co.verify_strict_many(msgs, pks, sigs, 1).sum()) == 0

        own = []
        el = bench.timed_steps(step, args.steps, args.warmup, world, dist, lambda: None, local_out=own)
        ranks = bench.gather_ranks({"rank": rank, "device": local, "pci_bus": None, "index_range": [lo, hi],
                                    "verify_per_s": round(n * args.steps / own[0], 1), "verdicts_ok": ok[0]},
                                   world, dist)
        if rank == 0:
            base = {"metric": "ed25519 verifications/sec", "value": round(n * world * args.steps / el, 1),
                    "unit": "verifications/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                    "ms_per_step": round(el / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
                    "vs_baseline": None, "dtype": "u32", "data": "CPU oracle stand-in (test)",
                    "config": {"workload": "stand-in", "triples_per_gpu": n},
                    "verdicts_ok": all(r["verdicts_ok"] for r in ranks)}
            roof = {"bound": "valu-int32", "achieved": None, "peak": bench.PEAK_INT32_TOPS, "unit": "TOPS",
                    "frac": None, "traffic": None}
            print(json.dumps(bench.headline(base, roof, None, {"c2_verify_per_s": base["value"]}, ranks=ranks)),
                  flush=True)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
