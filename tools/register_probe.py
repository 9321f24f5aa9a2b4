"""Probe: what a committee re-registration does to the aggregation queue's
windows.  A paced certificate stream (committee 100, C3 certificates, one
coa_queue_submit_certificate each, tools/latc.c latc_paced) runs on one
thread while another re-registers the same committee twice
(COA_REGISTER_TRACE=1 prints each registration's phases on stderr).  Prints
one JSON line: the registration windows (start/end, s from the stream's
start), the slowest requests (arrival, latency) and the latency percentiles
inside and outside the registrations.

usage: python tools/register_probe.py [rate_per_s] [seconds] [registrations] [reopen]
(reopen = 1: shut the engine down and re-open it with eight contexts, then
with one, and register a committee of 12 first -- the order of
tests/test_gpu_recovery.py run on its own)"""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xrpl-coa-prototype_amd"))
sys.path.insert(0, ROOT)


def main():
    rate = float(sys.argv[1]) if len(sys.argv) > 1 else 5000.0
    seconds = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
    n_reg = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    os.environ["COA_REGISTER_TRACE"] = "1"
    os.environ["COA_QUEUE_IDLE_LAUNCH"] = "1"
    import numpy as np
    import torch  # noqa: F401  (one HIP runtime: torch's)

    import bench
    import certificates as C
    import coa_crypto

    coa_crypto.init(0)
    if len(sys.argv) > 4 and sys.argv[4] == "1":
        coa_crypto.shutdown()
        coa_crypto.init_devices([0] * 8)
        coa_crypto.shutdown()
        coa_crypto.init(0)
        small, _ = C.synth_certificates(4, committee_size=12, n_payload=3, seed=31)
        for _ in range(3):
            coa_crypto.committee_register(np.zeros((0, 32), np.uint8))
            small.register()
    committee, certs = C.synth_certificates(100, committee_size=100, n_payload=32, seed=41)
    committee.register()
    n = int(rate * seconds)
    arrive = np.arange(n) / rate
    regs = []
    t_start = [0.0]

    def registrar():
        time.sleep(0.6)
        for _ in range(n_reg):
            a = time.monotonic() - t_start[0]
            committee.register()
            regs.append((a, time.monotonic() - t_start[0]))
            time.sleep(0.4)

    th = threading.Thread(target=registrar)
    t_start[0] = time.monotonic()
    th.start()
    lat, el, met = bench.paced_queue(arrive, np.ones(n, np.int32), np.arange(n) % len(certs), certs=certs,
                                     cexp=np.zeros(len(certs), np.uint8), max_batch=4096, max_delay_us=200)
    th.join()
    during = np.zeros(n, bool)
    for a, b in regs:
        during |= (arrive >= a) & (arrive <= b)
    worst = np.argsort(-lat)[:12]
    out = {"rate": rate, "requests": n, "registrations_s": [[round(a, 3), round(b, 3)] for a, b in regs],
           "worst": [[round(float(arrive[i]), 4), round(float(lat[i]), 3)] for i in worst],
           "p99_ms_during": round(float(np.percentile(lat[during], 99)), 3) if during.any() else None,
           "p99_ms_outside": round(float(np.percentile(lat[~during], 99)), 3),
           "max_ms_during": round(float(lat[during].max()), 3) if during.any() else None,
           "window_ms_max": round(met["window_us_max"] * 1e-3, 3), "window_max_items": int(met["window_max_items"]),
           "windows": int(met["windows"]), "max_in_flight": int(met["max_in_flight"]),
           "slot_wait_ms_max": round(met["slot_wait_us_max"] * 1e-3, 3), "staging_grows": int(met["staging_grows"]),
           "max_ms_per_100ms": [round(float(lat[(arrive >= b / 10) & (arrive < (b + 1) / 10)].max()), 2)
                                for b in range(int(seconds * 10))]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
