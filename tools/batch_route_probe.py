"""Where should verify_batch switch from the per-vote path (coa_batch.hip) to
the Pippenger path (coa_msm.hip)?  Times ONE group of n signatures through
coa_ed25519_verify_batch_groups (host buffers, as the Rust shim calls it)
with COA_MSM_MIN forcing each route, and both routes' verdicts on a corrupted
copy.

usage: python tools/batch_route_probe.py [n ...]   (default 1024 .. 262144)
An argument GxV times G groups of V signatures each (one message per group)
under both routings (COA_MSM_MIN=0: per-vote; unset: the default), e.g. 2x67
or 10000x67 (a C3 round with uncached keys).
Prints one JSON line per size."""
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


def timed(msg, pk, sg, offs, reps):
    coa_crypto.verify_batch_groups(msg, pk, sg, offs, rng_seed=7)
    t0 = time.perf_counter()
    for _ in range(reps):
        v = coa_crypto.verify_batch_groups(msg, pk, sg, offs, rng_seed=7)
    return (time.perf_counter() - t0) / reps * 1e3, int(v[0])


def groups(dev, ng, nv):
    """G groups of V signatures each, timed under both routings: COA_MSM_MIN=0
    (every group through one per-vote launch) and the default routing (calls
    with one or two groups, and groups >= 16,384, take the Pippenger path).
    Each row records the route and the COA_MSM_MIN it ran under, and checks
    that a corrupted copy (one flipped s bit in the last group) is rejected."""
    n = ng * nv
    gm = messages(ng)
    m = torch.from_numpy(np.repeat(gm, nv, axis=0)).to(dev)
    seeds = torch.from_numpy(key_seeds(n)).to(dev)
    pk = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    sg = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    coa_crypto.sign_many_device(0, seeds, m, pk, sg)
    torch.cuda.synchronize()
    pk, sg = pk.cpu().numpy(), sg.cpu().numpy()
    bad = sg.copy()
    bad[n - 1, 40] ^= 1
    offs = np.arange(ng + 1, dtype=np.uint64) * nv
    row = {"groups": ng, "votes_per_group": nv}
    for mmin in ("0", None):
        if mmin is None:
            os.environ.pop("COA_MSM_MIN", None)
            route = "pippenger" if (ng <= 2 or nv >= 16384) else "per_vote"
            label = "default"
        else:
            os.environ["COA_MSM_MIN"] = mmin
            route, label = "per_vote", "msm_min_0"
        coa_crypto.verify_batch_groups(gm, pk, sg, offs, rng_seed=7)
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            v = coa_crypto.verify_batch_groups(gm, pk, sg, offs, rng_seed=7)
        ms = (time.perf_counter() - t0) / reps * 1e3
        vb = coa_crypto.verify_batch_groups(gm, pk, bad, offs, rng_seed=7)
        row[label] = {"route": route, "COA_MSM_MIN": mmin if mmin is not None else "unset (16384)",
                      "ms": round(ms, 4), "groups_per_s": round(ng / ms * 1e3, 1),
                      "sig_per_s": round(n / ms * 1e3, 1), "valid_ok": int(v.sum()) == 0,
                      "corrupt_rejected": int(vb[-1]) == 1 and int(vb[:-1].sum()) == 0}
    os.environ.pop("COA_MSM_MIN", None)
    print(json.dumps(row), flush=True)


def main():
    sizes = [tuple(int(x) for x in a.split("x")) if "x" in a else int(a) for a in sys.argv[1:]] or [1024, 4096, 8192, 16384, 32768, 65536, 262144]
    coa_crypto.init(1)
    dev = torch.device("cuda", 0)
    for n in sizes:
        if isinstance(n, tuple):
            groups(dev, *n)
            continue
        m = torch.from_numpy(np.tile(messages(1), (n, 1))).to(dev)
        seeds = torch.from_numpy(key_seeds(n)).to(dev)
        pk = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        sg = torch.empty((n, 64), dtype=torch.uint8, device=dev)
        coa_crypto.sign_many_device(0, seeds, m, pk, sg)
        torch.cuda.synchronize()
        msg, pk, sg = m[:1].cpu().numpy(), pk.cpu().numpy(), sg.cpu().numpy()
        bad = sg.copy()
        bad[n // 3, 40] ^= 1
        offs = np.array([0, n], np.uint64)
        reps = 20 if n <= 65536 else 5
        row = {"n": n}
        for route, mmin in (("per_vote", "0"), ("pippenger", "1")):
            os.environ["COA_MSM_MIN"] = mmin
            ms, ok = timed(msg, pk, sg, offs, reps)
            _, bad_v = timed(msg, pk, bad, offs, 1)
            row[route] = {"ms": round(ms, 4), "sig_per_s": round(n / ms * 1e3, 1), "valid_ok": ok == 0,
                          "corrupt_rejected": bad_v == 1}
        print(json.dumps(row), flush=True)
    os.environ.pop("COA_MSM_MIN", None)


if __name__ == "__main__":
    main()
