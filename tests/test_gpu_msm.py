"""GPU parity of the Pippenger batch equation (csrc/coa_msm.hip):
crypto::Signature::verify_batch (crypto/src/lib.rs:206-219) -> dalek 1.0.1
verify_batch over one large group.  With explicit weights z_i the
multiscalar sum is exact, so the verdict must equal the oracle's (small
groups) and the per-vote path's (coa_batch.hip, large groups) bit for bit,
torsion components included.  COA_MSM_MIN (read per call) routes groups of
at least that many signatures to the Pippenger kernels; COA_MSM_RUN picks the
bucket workgroup's run length (16, 32, 64 sorted points per lane).
COA_BATCH_LAT=0 keeps small calls off the latency prefilter
(test_gpu_batch.py covers that route)."""
import random
import struct

import numpy as np
import pytest

import ed25519_ref as o
from conftest import load_golden
from test_gpu_batch import _pack

pytestmark = pytest.mark.gpu


def _torsion8():
    for T in o.torsion_points():
        if not o.is_identity(o.pdbl(o.pdbl(T))):
            return T
    raise AssertionError


def _mixed_vote(seed, m, T8, rng):
    """(pk, sig, j, k) with a mixed-order key A = aB + T8 and R = rB + jT8
    whose torsion part cancels in verify_strict's equation (j + k = 0 mod 8).
    In a batch the vote adds z j T8 + (z k mod l) T8, so the batch verdict
    is Ok iff z j + (z k mod l) = 0 mod 8."""
    a, _ = o.expand_seed(seed)
    Ab = o.compress(o.padd(o.pmul(a, o.B), T8))
    while True:
        r = rng.getrandbits(256) % o.L
        for j in range(8):
            Rb = o.compress(o.padd(o.pmul(r, o.B), o.pmul(j, T8)))
            k = o.scalar_from_hash(o.sha512(Rb + Ab + m))
            if (j + k) % 8 == 0:
                return Ab, Rb + ((r + k * a) % o.L).to_bytes(32, "little"), j, k


def _signed(engine, n, tag):
    from workloads import key_seeds

    seeds = key_seeds(n)
    m = o.sha512(b"msm" + tag)[:32]
    pks, sigs = engine.sign_many(seeds, np.tile(np.frombuffer(m, np.uint8), (n, 1)))
    return m, pks, sigs


def _verdicts(engine, monkeypatch, msm_min, msgs, pks, sigs, offs, zs=None, run=None, seed=0):
    # the exact kernels themselves, not the latency prefilter of small calls
    monkeypatch.setenv("COA_BATCH_LAT", "0")
    monkeypatch.setenv("COA_MSM_MIN", str(msm_min))
    if run is None:
        monkeypatch.delenv("COA_MSM_RUN", raising=False)
    else:
        monkeypatch.setenv("COA_MSM_RUN", str(run))
    return engine.verify_batch_groups(msgs, pks, sigs, offs, zs=zs, rng_seed=seed)


def test_golden_batch_vectors_via_msm(engine, monkeypatch):
    """Every golden verify_batch group through the Pippenger kernels."""
    gs = []
    for g in load_golden("batch_vectors.json"):
        gs.append({"msg": bytes.fromhex(g["msg"]), "pks": [bytes.fromhex(p) for p in g["pks"]],
                   "sigs": [bytes.fromhex(s) for s in g["sigs"]], "zs": [int(z, 16) for z in g["zs"]],
                   "expect": g["expect"], "name": g["name"]})
    msgs, pks, sigs, offs, zs = _pack(gs)
    got = _verdicts(engine, monkeypatch, 1, msgs, pks, sigs, offs, zs=zs)
    bad = [g["name"] for g, v in zip(gs, got) if (v == 0) != g["expect"]]
    assert not bad, bad


def test_torsion_groups_exact_via_msm(engine, monkeypatch):
    """Mixed-order keys: both verdicts occur, each equal to the oracle's for
    the same z (the torsion part survives iff 8 does not divide sum z_i k_i)."""
    rng = random.Random(11)
    T8 = _torsion8()
    groups = []
    for gi in range(10):
        m = o.sha512(b"msm-tors" + bytes([gi]))[:32]
        seeds = [o.sha512(b"coa-key" + struct.pack("<Q", 900 + gi * 5 + j))[:32] for j in range(5)]
        pks = [o.public_key(s) for s in seeds]
        sigs = [o.sign(s, m) for s in seeds]
        pks[2], sigs[2], _, _ = _mixed_vote(seeds[2], m, T8, rng)
        zs = [rng.getrandbits(128) for _ in range(5)]
        groups.append({"msg": m, "pks": pks, "sigs": sigs, "zs": zs, "expect": o.verify_batch(m, pks, sigs, zs)})
    assert any(g["expect"] for g in groups) and not all(g["expect"] for g in groups)
    msgs, pks, sigs, offs, zs = _pack(groups)
    got = _verdicts(engine, monkeypatch, 1, msgs, pks, sigs, offs, zs=zs)
    assert [v == 0 for v in got] == [g["expect"] for g in groups]


@pytest.mark.parametrize("run,tree,pstride", [(16, 1, 32), (32, 1, 32), (64, 1, 32), (16, 0, 32), (64, 0, 24),
                                              (32, 1, 24), (4, 1, 32), (4, 0, 32)])
def test_large_group_matches_per_vote_path(engine, monkeypatch, run, tree, pstride):
    """n = 20,011 (odd point counts across chunk boundaries at every run):
    valid, one corrupted s, one non-canonical s, one undecodable R, and equal
    weights (every R_i digit in one bucket: a bucket spanning all lanes).
    Both forms of the window sums (COA_MSM_TREE: per chunk, or buckets summed
    over chunks first) and both point-record strides (COA_MSM_PSTRIDE).  At
    run 4 (1,024 points per chunk) 19 of the 40 chunks hold R points only and
    get no workgroup in windows 15..28, across the tree groups' boundaries."""
    monkeypatch.setenv("COA_MSM_TREE", str(tree))
    monkeypatch.setenv("COA_MSM_PSTRIDE", str(pstride))
    n = 20011
    m, pks, sigs = _signed(engine, n, b"large")
    msgs = np.frombuffer(m, np.uint8).reshape(1, 32).copy()
    offs = np.array([0, n], np.uint64)
    rng = np.random.default_rng(3)
    zs = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    cases = {"valid": (pks, sigs, zs)}
    s1 = sigs.copy()
    s1[n // 2, 40] ^= 4
    cases["corrupt"] = (pks, s1, zs)
    s2 = sigs.copy()
    s2[7, 32:] = np.frombuffer((o.L + 1).to_bytes(32, "little"), np.uint8)
    cases["s_noncanonical"] = (pks, s2, zs)
    s3 = sigs.copy()
    s3[n - 1, :32] = np.frombuffer(bytes.fromhex("02" + "00" * 31), np.uint8)  # y = 2: not on the curve
    cases["r_undecodable"] = (pks, s3, zs)
    cases["equal_weights"] = (pks, sigs, np.tile(zs[:1], (n, 1)))
    cases["zero_weights_corrupt"] = (pks, s1, np.zeros_like(zs))
    for name, (p, s, z) in cases.items():
        ref = _verdicts(engine, monkeypatch, 0, msgs, p, s, offs, zs=z)
        got = _verdicts(engine, monkeypatch, 1024, msgs, p, s, offs, zs=z, run=run)
        assert got[0] == ref[0], (name, got, ref)
        assert (got[0] == 0) == (name in ("valid", "equal_weights", "zero_weights_corrupt")), name


@pytest.mark.parametrize("n", [1, 67, 300, 511, 512, 1000, 2047])
def test_one_chunk_groups_short_runs(engine, monkeypatch, n):
    """Groups that fit one bucket workgroup take runs of 4..16 sorted points
    per lane (n = 511 / 512: 1,023 / 1,025 points, either side of run 4's
    1,024): valid, a corrupted vote and equal weights agree with the
    per-vote path."""
    m, pks, sigs = _signed(engine, n, b"short" + bytes([n & 255]))
    msgs = np.frombuffer(m, np.uint8).reshape(1, 32).copy()
    offs = np.array([0, n], np.uint64)
    zs = np.random.default_rng(n).integers(0, 256, (n, 16), dtype=np.uint8)
    bad = sigs.copy()
    bad[n // 2, 50] ^= 16
    for name, s_, z in (("valid", sigs, zs), ("corrupt", bad, zs), ("equal", sigs, np.tile(zs[:1], (n, 1)))):
        ref = _verdicts(engine, monkeypatch, 0, msgs, pks, s_, offs, zs=z)
        got = _verdicts(engine, monkeypatch, 1, msgs, pks, s_, offs, zs=z)
        assert got[0] == ref[0] == (1 if name == "corrupt" else 0), (n, name, got, ref)


def test_large_group_with_torsion_vote(engine, monkeypatch):
    """A mixed-order vote inside a 4,099-signature batch, with its weight
    chosen so the torsion part cancels (Ok) or survives (Err): the Pippenger
    verdict equals the per-vote path's and the expected one."""
    rng = random.Random(17)
    T8 = _torsion8()
    n = 4099
    m, pks, sigs = _signed(engine, n, b"tors-large")
    from workloads import key_seeds

    seed0 = bytes(key_seeds(1)[0])
    pk, sg, j, k = _mixed_vote(seed0, m, T8, rng)
    pks = pks.copy()
    sigs = sigs.copy()
    pks[0] = np.frombuffer(pk, np.uint8)
    sigs[0] = np.frombuffer(sg, np.uint8)
    msgs = np.frombuffer(m, np.uint8).reshape(1, 32).copy()
    offs = np.array([0, n], np.uint64)
    for trial in range(6):
        want_ok = trial % 2 == 0
        while True:
            z0 = rng.getrandbits(128)
            if ((z0 * j + (z0 * k) % o.L) % 8 == 0) == want_ok:
                break
        zs = np.frombuffer(bytes(rng.getrandbits(8) for _ in range(16 * n)), np.uint8).reshape(n, 16).copy()
        zs[0] = np.frombuffer(z0.to_bytes(16, "little"), np.uint8)
        ref = _verdicts(engine, monkeypatch, 0, msgs, pks, sigs, offs, zs=zs)
        got = _verdicts(engine, monkeypatch, 64, msgs, pks, sigs, offs, zs=zs)
        assert got[0] == ref[0] == (0 if want_ok else 1), (trial, got, ref)


def test_mixed_sizes_route_and_agree(engine, monkeypatch):
    """Large and small groups in one call: each large group goes through the
    Pippenger path, runs of small ones through the per-vote path; verdicts
    equal the all-per-vote call's."""
    sizes = [3, 5000, 67, 67, 6000, 0, 4]
    n = sum(sizes)
    m, pks, sigs = _signed(engine, n, b"mixed")
    offs = np.zeros(len(sizes) + 1, np.uint64)
    offs[1:] = np.cumsum(sizes)
    msgs = np.tile(np.frombuffer(m, np.uint8), (len(sizes), 1))
    sigs = sigs.copy()
    sigs[int(offs[4]) + 10, 50] ^= 1   # group 4 (large) fails
    sigs[int(offs[2]) + 1, 50] ^= 1    # group 2 (small) fails
    rng = np.random.default_rng(5)
    zs = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    ref = _verdicts(engine, monkeypatch, 0, msgs, pks, sigs, offs, zs=zs)
    got = _verdicts(engine, monkeypatch, 1000, msgs, pks, sigs, offs, zs=zs)
    assert list(got) == list(ref) == [0, 0, 1, 0, 1, 0, 0]
    # seeded weights: all torsion-free, so the verdicts do not depend on z
    got2 = _verdicts(engine, monkeypatch, 1000, msgs, pks, sigs, offs, seed=99)
    assert list(got2) == list(ref)


def test_device_entry_resident(engine):
    """coa_ed25519_verify_batch_device on HBM-resident tensors (the bench
    path): 65,536 device-signed votes, seeded and explicit weights."""
    import torch

    from workloads import key_seeds, messages

    n = 65536
    dev = torch.device("cuda", 0)
    m = torch.from_numpy(np.tile(messages(1), (n, 1))).to(dev)
    seeds = torch.from_numpy(key_seeds(n)).to(dev)
    pk = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    sg = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    engine.sign_many_device(0, seeds, m, pk, sg)
    msg = m[0].contiguous()
    out = torch.full((1,), 7, dtype=torch.uint8, device=dev)
    ws = torch.empty(engine.verify_batch_workspace_bytes(n), dtype=torch.uint8, device=dev)
    engine.verify_batch_device(0, msg, pk, sg, out, rng_seed=1, workspace=ws)
    torch.cuda.synchronize()
    assert int(out[0]) == 0
    zs = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device=dev)
    sg[12345, 33] ^= 1
    engine.verify_batch_device(0, msg, pk, sg, out, zs=zs)
    torch.cuda.synchronize()
    assert int(out[0]) == 1
    sg[12345, 33] ^= 1
    engine.verify_batch_device(0, msg, pk, sg, out, zs=zs)
    torch.cuda.synchronize()
    assert int(out[0]) == 0
    engine.verify_batch_device(0, msg, pk[:0], sg[:0], out, rng_seed=1)  # empty batch: Ok
    torch.cuda.synchronize()
    assert int(out[0]) == 0
    # a workspace smaller than verify_batch_workspace_bytes(n) is refused
    with pytest.raises(engine.EngineError):
        engine.verify_batch_device(0, msg, pk, sg, out, rng_seed=1, workspace=ws[:4096])


@pytest.mark.parametrize("n", [600_000, 1 << 21])
def test_large_groups_resident(engine, n):
    """Large groups (2^21 at run 64: 128 of 257 chunks hold R points alone
    and get no workgroups in windows 15..28) on HBM-resident votes: valid
    with seeded and with equal weights (every R_i digit in one bucket), and
    one corrupted s in an R-only chunk, in the chunk where the A points
    start and in the last vote, each an Err."""
    import torch

    from workloads import key_seeds, messages

    dev = torch.device("cuda", 0)
    m = torch.from_numpy(np.tile(messages(1), (n, 1))).to(dev)
    seeds = torch.from_numpy(key_seeds(n)).to(dev)
    pk = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    sg = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    engine.sign_many_device(0, seeds, m, pk, sg)
    del seeds
    msg = m[0].contiguous()
    del m
    out = torch.full((1,), 7, dtype=torch.uint8, device=dev)
    ws = torch.empty(engine.verify_batch_workspace_bytes(n), dtype=torch.uint8, device=dev)
    engine.verify_batch_device(0, msg, pk, sg, out, rng_seed=3, workspace=ws)
    torch.cuda.synchronize()
    assert int(out[0]) == 0
    zs = torch.randint(0, 256, (1, 16), dtype=torch.uint8, device=dev).repeat(n, 1)
    engine.verify_batch_device(0, msg, pk, sg, out, zs=zs, workspace=ws)
    torch.cuda.synchronize()
    assert int(out[0]) == 0
    for i in (5, n // 2 - 3, n - 1):
        sg[i, 40] ^= 2
        engine.verify_batch_device(0, msg, pk, sg, out, rng_seed=4, workspace=ws)
        torch.cuda.synchronize()
        assert int(out[0]) == 1, i
        sg[i, 40] ^= 2
