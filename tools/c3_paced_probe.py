"""Streamed C3 paced from 4 producers, repeated: achieved rate, wait p50/p99,
this process's CPU use and the cgroup's CPU throttling per run (bench.py's
c3_stream, one configuration at a time).  Prints the cgroup's cpu.max first.

  python tools/c3_paced_probe.py [--rates 3000000,2000000] [--reps 4] [--burst 4]

Question it answers: is the paced-3M tail (p99 ~8 ms, achieved ~2.4 M/s in
round 6's bench runs) the engine, or the process running out of its CPU
quota (a throttled period stalls every thread for the rest of the period)."""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rates", default="3000000")
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--burst", default="", help="producer counts for burst runs (borrowed), e.g. 4,8")
    a = ap.parse_args()
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "/sys/fs/cgroup/cpu/cpu.cfs_period_us"):
        try:
            print(path, open(path).read().strip())
        except OSError:
            pass
    print("sched_getaffinity", len(os.sched_getaffinity(0)), flush=True)
    import certificates as C
    import coa_crypto

    coa_crypto.init_devices([0])
    lib = bench._latc()
    vp, sz, ci, dp = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_double)
    lib.latc_stream_certificates.argtypes = [sz, ctypes.c_uint, ci, ci, ci, ctypes.c_double] + [vp] * 9 + [sz, vp, dp,
                                                                                                          vp]
    lib.latc_stream_certificates.restype = ci
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
    expect = np.zeros(n_certs, np.uint8)
    ptrs = [x.ctypes.data for x in arrs]
    rates = [int(r) for r in a.rates.split(",") if r]
    burst = [int(p) for p in a.burst.split(",") if p]
    for rep in range(a.reps):
        if burst:
            r = bench.c3_stream(lib, ptrs, n_certs, expect, producer_counts=burst, borrowed_modes=(1,), rates=())
            for k, v in r.items():
                if k != "mode":
                    print(json.dumps({"rep": rep, "run": k, "certs_per_s": v["certs_per_s"], "p50": v["wait_ms_p50"],
                                      "p99": v["wait_ms_p99"], "host": v["diag"]["host"],
                                      "stages": v["diag"]["stage_us_per_window"]}), flush=True)
        r = bench.c3_stream(lib, ptrs, n_certs, expect, producer_counts=(), rates=rates)
        for k, v in r.items():
            if k != "mode":
                print(json.dumps({"rep": rep, "run": k, "achieved": v["achieved_certs_per_s"], "p50": v["wait_ms_p50"],
                                  "p99": v["wait_ms_p99"], "host": v["diag"]["host"],
                                  "window_ms_max": v["diag"]["window_ms_max"],
                                  "stages": v["diag"]["stage_us_per_window"]}), flush=True)
    coa_crypto.committee_register(np.zeros((0, 32), np.uint8))


if __name__ == "__main__":
    main()
