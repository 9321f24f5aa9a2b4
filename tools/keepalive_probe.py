"""Probe (round 5): is the queue's low-rate latency (C1 round mix at 10
rounds/s: p50 ~0.07 ms against ~0.047 at 1,000 rounds/s) the GPU leaving its
busy clocks between sparse requests?  Runs bench.queue_round_mix for the C1
committee at 10 and 1,000 rounds/s (idle launch) alternately without and with
a background thread that keeps the GPU busy with one tiny kernel every
`period_us` on its own stream.  Diagnostics only; prints JSON lines."""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    import coa_crypto

    coa_crypto.init_devices([0])
    period_us = float(sys.argv[1]) if len(sys.argv) > 1 else 500.0
    stop = threading.Event()

    def keepalive():
        s = torch.cuda.Stream()
        x = torch.zeros(64, device="cuda")
        with torch.cuda.stream(s):
            while not stop.is_set():
                x.add_(1.0)
                time.sleep(period_us * 1e-6)

    for rep in range(2):
        for ka in (False, True):
            th = None
            if ka:
                stop.clear()
                th = threading.Thread(target=keepalive, daemon=True)
                th.start()
                time.sleep(0.05)
            r = bench.queue_round_mix(rates=(10, 1000), committee_size=4, n_payload=1)
            if th:
                stop.set()
                th.join()
            out = {"rep": rep, "keepalive_us": period_us if ka else None}
            for rate, row in r["rates_idle_launch"].items():
                out[rate] = {k: [row[k]["p50_ms"], row[k]["p99_ms"]] for k in ("certificate", "signature")}
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
