"""Latency of ONE uncached verify_batch group (one certificate's 67 votes,
host pointers in, verdict out: Signature::verify_batch, crypto/src/lib.rs:
206-219) -- p50 over `calls` calls; under `rocprofv3 --kernel-trace` the
trace shows how the call's wall time splits into kernels and gaps.

usage: python tools/msm1_probe.py [votes] [calls] [groups]
(groups > 1: that many certificates of `votes` votes each in one call)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xrpl-coa-prototype_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import coa_crypto  # noqa: E402
from workloads import key_seeds, messages  # noqa: E402

nv = int(sys.argv[1]) if len(sys.argv) > 1 else 67
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 200
ng = int(sys.argv[3]) if len(sys.argv) > 3 else 1
coa_crypto.init(0)
msg = messages(ng, 4242)
m = np.repeat(msg, nv, axis=0)
pks, sigs = coa_crypto.sign_many(key_seeds(nv * ng, 9000), m)
offs = np.arange(0, nv * ng + 1, nv, dtype=np.uint64)
lat = []
for i in range(calls + 20):
    t0 = time.perf_counter()
    v = coa_crypto.verify_batch_groups(msg, pks, sigs, offs)
    lat.append(time.perf_counter() - t0)
    assert not v.any()
lat = np.array(lat[20:]) * 1e3
print(json.dumps({"votes": nv, "groups": ng, "route": os.environ.get("COA_BATCH_LAT", "default"), "calls": calls,
                  "p50_ms": round(float(np.percentile(lat, 50)), 4),
                  "p99_ms": round(float(np.percentile(lat, 99)), 4)}))
