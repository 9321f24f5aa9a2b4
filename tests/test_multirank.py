"""CPU, world_size 2 (gloo): the N>1 path of bench.py and of the library's
host-call sharding -- disjoint contiguous index ranges that cover the global
set, per-rank verification with no data-path collective, verdicts reassembled
in place, max-over-ranks timing.  The per-rank verifier here is the CPU oracle
(test infrastructure), standing in for each rank's GPU."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import sharding


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_per_rank, q):
    import torch

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import coa_oracle as co
        import workloads

        lo, hi = sharding.rank_slice(rank, world, n_per_rank)
        seeds = workloads.key_seeds(hi - lo, start=lo)
        msgs = workloads.messages(hi - lo, start=lo)
        # valid triples from the Python oracle are slow; use a tiny n
        import ed25519_ref as o

        pks = np.frombuffer(b"".join(o.public_key(bytes(s)) for s in seeds), np.uint8).reshape(-1, 32).copy()
        sigs = np.frombuffer(b"".join(o.sign(bytes(s), bytes(m)) for s, m in zip(seeds, msgs)),
                             np.uint8).reshape(-1, 64).copy()
        sigs[::5, 40] ^= 1  # every 5th local item invalid
        v = co.verify_strict_many(msgs, pks, sigs, 1)
        gathered = [torch.zeros(hi - lo, dtype=torch.uint8) for _ in range(world)]
        dist.all_gather(gathered, torch.from_numpy(v))
        ranges = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(ranges, torch.tensor([lo, hi]))
        t = sharding.max_over_ranks(float(rank + 1), dist)
        if rank == 0:
            q.put((np.concatenate([g.numpy() for g in gathered]), [r.tolist() for r in ranges], t))
    finally:
        dist.destroy_process_group()


def test_two_rank_weak_scaling_path():
    world, n_per_rank = 2, 12
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_per_rank, q)) for r in range(world)]
    for p in procs:
        p.start()
    verdicts, ranges, t = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert ranges == [[0, 12], [12, 24]]  # disjoint, contiguous, covering
    expect = np.array([1 if (i % n_per_rank) % 5 == 0 else 0 for i in range(world * n_per_rank)], np.uint8)
    assert (verdicts == expect).all()
    assert t == 2.0  # max over ranks


@pytest.mark.parametrize("n,parts", [(0, 8), (1, 8), (7, 8), (65536, 8), (16_777_216, 8), (10, 3)])
def test_shard_ranges_cover(n, parts):
    rs = sharding.shard_ranges(n, parts)
    covered = sum(hi - lo for _, lo, hi in rs)
    assert covered == n
    for (_, a, b), (_, c, d) in zip(rs, rs[1:]):
        assert b == c
    if n >= parts:
        sizes = [hi - lo for _, lo, hi in rs]
        assert max(sizes) - min(sizes) <= 1


def _bench_rank(rank, world, port, q):
    """One rank of bench.py's timed region (bench.timed_steps): gloo barrier
    on both sides, max-over-ranks elapsed.  Rank r's step verifies its own
    contiguous slice with the CPU oracle (standing in for its GPU) and sleeps
    r * 30 ms per step, so the max must be rank 1's time."""
    import time

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        import coa_oracle as co
        import ed25519_ref as o
        import workloads

        n = 6
        lo, hi = sharding.rank_slice(rank, world, n)
        seeds, msgs = workloads.key_seeds(n, start=lo), workloads.messages(n, start=lo)
        pks = np.frombuffer(b"".join(o.public_key(bytes(s)) for s in seeds), np.uint8).reshape(-1, 32).copy()
        sigs = np.frombuffer(b"".join(o.sign(bytes(s), bytes(m)) for s, m in zip(seeds, msgs)),
                             np.uint8).reshape(-1, 64).copy()
        calls = []

        def step(i):
            v = co.verify_strict_many(msgs, pks, sigs, 1)
            assert int(v.sum()) == 0
            time.sleep(0.03 * rank)
            calls.append(i)

        t0 = time.perf_counter()
        el = bench.timed_steps(step, 4, 2, world, dist, lambda: None)
        own = time.perf_counter() - t0
        q.put((rank, el, own, calls))
    finally:
        dist.destroy_process_group()


def test_bench_timed_region_two_ranks():
    """bench.py's own rank path (timed_steps) under world 2: warmup steps are
    untimed (step(None)), exactly `steps` timed steps, the reported time is the
    max over ranks and identical on both ranks, and it covers the slow rank's
    sleeps."""
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if root not in sys.path:
        sys.path.insert(0, root)
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, el0, _, calls0), (_, el1, _, calls1) = res
    assert el0 == el1                   # one max, seen by every rank
    assert el1 >= 4 * 0.03              # includes rank 1's four timed sleeps
    assert calls0 == calls1 == [None, None, 0, 1, 2, 3]
