"""Single-signature latency route (coa_latency.hip) on the GPU box:
  * p50/p99 of one Signature::verify per call (host pointers in, verdict out)
    with the key outside / inside the registered committee;
  * a sweep over call sizes n: wall time of coa_ed25519_verify_strict_many
    through the latency kernel (COA_LAT_MAX large) and through the split
    throughput kernels (COA_LAT_MAX=0) -- where the route should switch.
Prints one JSON line per measurement."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xrpl-coa-prototype_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (HIP runtime shared with torch)

import coa_crypto  # noqa: E402
from workloads import key_seeds, messages  # noqa: E402


def p(lat):
    a = np.array(lat) * 1e3
    return round(float(np.percentile(a, 50)), 4), round(float(np.percentile(a, 99)), 4)


def main():
    coa_crypto.init(1)
    n0 = 64
    seeds, msgs = key_seeds(n0, 777), messages(n0, 777)
    pks, sigs = coa_crypto.sign_many(seeds, msgs)
    for label, reg in (("uncached", False), ("cached", True)):
        coa_crypto.committee_register(pks if reg else np.zeros((0, 32), np.uint8))
        lat = []
        for i in range(1200):
            j = i % n0
            sg = coa_crypto.Signature.from_bytes(bytes(sigs[j]))
            d, pk = bytes(msgs[j]), bytes(pks[j])
            t0 = time.perf_counter()
            sg.verify(d, pk)
            lat.append(time.perf_counter() - t0)
        p50, p99 = p(lat[200:])
        print(json.dumps({"single_verify": label, "p50_ms": p50, "p99_ms": p99}), flush=True)
    coa_crypto.committee_register(np.zeros((0, 32), np.uint8))
    sizes = [int(x) for x in sys.argv[1:]] or [1, 4, 16, 64, 256, 1024, 2048, 4096]
    big = max(sizes)
    seeds, msgs = key_seeds(big, 5000), messages(big, 5000)
    pks, sigs = coa_crypto.sign_many(seeds, msgs)
    for n in sizes:
        row = {"n": n}
        for route, mx in (("latency", str(10 ** 9)), ("split", "0")):
            os.environ["COA_LAT_MAX"] = mx
            v = coa_crypto.verify_strict_many(msgs[:n], pks[:n], sigs[:n])
            assert int(v.sum()) == 0
            lat = []
            for _ in range(30):
                t0 = time.perf_counter()
                coa_crypto.verify_strict_many(msgs[:n], pks[:n], sigs[:n])
                lat.append(time.perf_counter() - t0)
            row[route + "_p50_ms"] = p(lat)[0]
        print(json.dumps(row), flush=True)
    os.environ.pop("COA_LAT_MAX", None)


if __name__ == "__main__":
    main()
