"""C2 throughput with several verify calls in flight (one stream and one
workspace per in-flight call, round-robin), as the aggregation queue runs its
double-buffered windows.  One line per in-flight depth:
  {"inflight": d, "n": 65536, "calls": K, "ms_per_call": ..., "verify_per_s": ...}

usage: python tools/inflight_probe.py [n] [calls]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xrpl-coa-prototype_amd"))


def main():
    import torch

    import coa_crypto
    import workloads

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    coa_crypto.init_devices([0])
    seeds = torch.from_numpy(workloads.key_seeds(n)).to(dev)
    msgs = torch.from_numpy(workloads.messages(n)).to(dev)
    pks = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    sigs = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    coa_crypto.sign_many_device(0, seeds, msgs, pks, sigs)
    torch.cuda.synchronize()
    for depth in (1, 2, 3, 4):
        streams = [torch.cuda.Stream(dev) for _ in range(depth)]
        wss = [torch.empty(coa_crypto.verify_workspace_bytes(n), dtype=torch.uint8, device=dev) for _ in range(depth)]
        outs = [torch.ones(n, dtype=torch.uint8, device=dev) for _ in range(depth)]

        def run(k):
            for i in range(k):
                j = i % depth
                coa_crypto.verify_strict_many_device(0, msgs, pks, sigs, outs[j], wss[j], streams[j])

        run(2 * depth)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(calls)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ok = all(int(o.sum().item()) == 0 for o in outs)
        print(json.dumps({"inflight": depth, "n": n, "calls": calls, "ms_per_call": round(dt / calls * 1e3, 4),
                          "verify_per_s": round(n * calls / dt, 1), "verdicts_ok": ok}), flush=True)


if __name__ == "__main__":
    main()
