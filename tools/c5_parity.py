"""C5 parity at full size (BASELINE.json configs[4]):
2^24 (digest, pk, sig) triples, 1% adversarial over the 8 classes (seeded
shuffle 0xC0A5), verified in 8 contiguous index-range shards (the per-GPU
slices of an 8-GPU node, run here one after another on the box's GPU) and
compared bit for bit with the C restatement of dalek (oracle/coa_oracle.c,
multithreaded).  Writes a JSON summary (argv[2], default
gpurun_out/c5_parity.json).

Inputs follow workloads.py's definitions (seed_i = SHA512("coa-key"||i)[..32],
M_i = SHA512(u64le i)[..32]); the hashing is done by the C oracle's SHA-512
so that generating 2 x 16M inputs takes seconds, not minutes."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xrpl-coa-prototype_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402


def log(*a):
    print(f"[{time.strftime('%H:%M:%S')}]", *a, flush=True)


def hashed_inputs(prefix, n, threads):
    import coa_oracle as co

    w = len(prefix) + 8
    buf = np.zeros((n, w), np.uint8)
    buf[:, :len(prefix)] = np.frombuffer(prefix, np.uint8)
    buf[:, len(prefix):] = np.arange(n, dtype="<u8").view(np.uint8).reshape(n, 8)
    offs = np.arange(n + 1, dtype=np.uint64) * w
    return co.sha512_many(buf.reshape(-1), offs, threads)[:, :32].copy()


def main():
    import coa_crypto
    import coa_oracle as co
    import workloads
    from conftest import load_golden

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 24
    out_path = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "c5_parity.json")
    shards = 8
    threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS", "16")), os.cpu_count() or 1, 64))
    coa_crypto.init(0)
    co.build()
    t0 = time.perf_counter()
    seeds = hashed_inputs(b"coa-key", n, threads)
    msgs = hashed_inputs(b"", n, threads)
    assert (seeds[:4] == workloads.key_seeds(4)).all() and (msgs[:4] == workloads.messages(4)).all()
    assert (seeds[-2:] == workloads.key_seeds(2, start=n - 2)).all()
    log(f"inputs hashed: {n} seeds + messages in {time.perf_counter() - t0:.1f} s")
    pks = np.empty((n, 32), np.uint8)
    sigs = np.empty((n, 64), np.uint8)
    step = 1 << 21
    for lo in range(0, n, step):
        p, s = coa_crypto.sign_many(seeds[lo:lo + step], msgs[lo:lo + step])
        pks[lo:lo + step], sigs[lo:lo + step] = p, s
    log("signed on device")
    pool = [(bytes.fromhex(v["msg"]), bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]))
            for v in load_golden("mixed_order_pool.json")]
    msgs, pks, sigs, cls = workloads.adversarial_mix(msgs, pks, sigs, frac=0.01, seed=0xC0A5, mixed_pool=pool)
    n_adv = int((cls >= 0).sum())
    log(f"adversarial mix: {n_adv} items over {len(np.unique(cls[cls >= 0]))} classes")
    got = np.empty(n, np.uint8)
    shard_ms = []
    for g in range(shards):
        lo, hi = n * g // shards, n * (g + 1) // shards
        t1 = time.perf_counter()
        got[lo:hi] = coa_crypto.verify_strict_many(msgs[lo:hi], pks[lo:hi], sigs[lo:hi])
        shard_ms.append(round((time.perf_counter() - t1) * 1e3, 1))
    log(f"engine verdicts: {int((got == 0).sum())} Ok, {int(got.sum())} Err; shard wall ms {shard_ms}")
    exp = np.empty(n, np.uint8)
    step = 1 << 20
    t2 = time.perf_counter()
    for lo in range(0, n, step):
        exp[lo:lo + step] = co.verify_strict_many(msgs[lo:lo + step], pks[lo:lo + step], sigs[lo:lo + step],
                                                  threads)
        if (lo // step) % 4 == 3:
            log(f"oracle {lo + step}/{n}")
    cpu_s = time.perf_counter() - t2
    mism = np.nonzero(got != exp)[0]
    per_class = {}
    for c, name in enumerate(workloads.ADVERSARIAL_CLASSES):
        m = cls == c
        per_class[name] = {"items": int(m.sum()), "accepted": int((exp[m] == 0).sum()),
                           "rejected": int((exp[m] == 1).sum())}
    res = {"config": "C5: 2^24 triples, 1% adversarial (seed 0xC0A5), 8 index-range shards on one GPU",
           "n": n, "adversarial": n_adv, "mismatches": int(mism.size),
           "mismatch_idx": [int(i) for i in mism[:20]], "bit_exact": bool(mism.size == 0),
           "untouched_all_ok": bool((got[cls == -1] == 0).all()), "per_class_oracle": per_class,
           "shard_wall_ms_host_api": shard_ms, "oracle_cpu_s": round(cpu_s, 1), "oracle_threads": threads}
    os.makedirs(os.path.dirname(out_path), exist_ok=True)
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    log(json.dumps({k: res[k] for k in ("n", "adversarial", "mismatches", "bit_exact", "untouched_all_ok")}))
    sys.exit(0 if mism.size == 0 else 1)


if __name__ == "__main__":
    main()
