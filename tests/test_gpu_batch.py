"""GPU parity: crypto::Signature::verify_batch (dalek 1.0.1 verify_batch) with
explicit weights z_i, so the multiscalar sum -- and hence the verdict -- is
the oracle's exactly, torsion components included."""
import random
import struct

import numpy as np
import pytest

import ed25519_ref as o
from conftest import load_golden

pytestmark = pytest.mark.gpu


def _pack(groups):
    msgs = np.frombuffer(b"".join(g["msg"] for g in groups), np.uint8).reshape(len(groups), 32).copy()
    pks = b"".join(p for g in groups for p in g["pks"])
    sigs = b"".join(s for g in groups for s in g["sigs"])
    zs = b"".join(z.to_bytes(16, "little") for g in groups for z in g["zs"])
    offs = np.zeros(len(groups) + 1, np.uint64)
    offs[1:] = np.cumsum([len(g["pks"]) for g in groups])
    n = int(offs[-1])
    return (msgs, np.frombuffer(pks, np.uint8).reshape(n, 32).copy(),
            np.frombuffer(sigs, np.uint8).reshape(n, 64).copy(), offs,
            np.frombuffer(zs, np.uint8).reshape(n, 16).copy())


@pytest.fixture(params=["prefilter", "exact"])
def route(request, monkeypatch):
    """Small calls through the latency prefilter (default) or straight to the
    exact batch kernels (COA_BATCH_LAT=0)."""
    monkeypatch.setenv("COA_BATCH_LAT", "1" if request.param == "prefilter" else "0")
    return request.param


def test_golden_batch_vectors(engine, route):
    gs = []
    for g in load_golden("batch_vectors.json"):
        gs.append({"msg": bytes.fromhex(g["msg"]), "pks": [bytes.fromhex(p) for p in g["pks"]],
                   "sigs": [bytes.fromhex(s) for s in g["sigs"]], "zs": [int(z, 16) for z in g["zs"]],
                   "expect": g["expect"], "name": g["name"]})
    msgs, pks, sigs, offs, zs = _pack(gs)
    got = engine.verify_batch_groups(msgs, pks, sigs, offs, zs=zs)
    bad = [g["name"] for g, v in zip(gs, got) if (v == 0) != g["expect"]]
    assert not bad, bad
    # seeded (engine-derived z) path agrees on these torsion-free groups
    got2 = engine.verify_batch_groups(msgs, pks, sigs, offs, rng_seed=12345)
    assert (got2 == got).all()


def _torsion_groups(seed=5):
    rng = random.Random(seed)
    T8 = None
    for T in o.torsion_points():
        if not o.is_identity(o.pdbl(o.pdbl(T))):
            T8 = T
            break
    groups = []
    for gi in range(12):
        m = o.sha512(b"tors" + bytes([gi]))[:32]
        seeds = [o.sha512(b"coa-key" + struct.pack("<Q", 500 + gi * 4 + j))[:32] for j in range(3)]
        pks = [o.public_key(s) for s in seeds]
        sigs = [o.sign(s, m) for s in seeds]
        # replace vote 0 by a mixed-order key with a torsion-matched R
        a, _ = o.expand_seed(seeds[0])
        A = o.padd(o.pmul(a, o.B), T8)
        Ab = o.compress(A)
        while True:
            r = rng.getrandbits(256) % o.L
            done = False
            for j in range(8):
                R = o.padd(o.pmul(r, o.B), o.pmul(j, T8))
                Rb = o.compress(R)
                k = o.scalar_from_hash(o.sha512(Rb + Ab + m))
                if (j + k) % 8 == 0:
                    pks[0] = Ab
                    sigs[0] = Rb + ((r + k * a) % o.L).to_bytes(32, "little")
                    done = True
                    break
            if done:
                break
        zs = [rng.getrandbits(128) for _ in range(3)]
        exp = o.verify_batch(m, pks, sigs, zs)
        groups.append({"msg": m, "pks": pks, "sigs": sigs, "zs": zs, "expect": exp})
    assert any(g["expect"] for g in groups) and not all(g["expect"] for g in groups)
    return groups


def test_torsion_batches_exact_with_given_z(engine, route):
    """Mixed-order A with a torsion-matched R passes verify_strict; in a batch
    the torsion part is multiplied by z_i h_i mod l, so the verdict depends
    on z -- both outcomes must match the oracle for the same z.  Through the
    prefilter the mixed-order key fails [l]A == O, so these groups are resolved
    by the exact kernels; a prefilter that accepted them would answer Ok for
    the groups the oracle rejects."""
    groups = _torsion_groups()
    msgs, pks, sigs, offs, zs = _pack(groups)
    got = engine.verify_batch_groups(msgs, pks, sigs, offs, zs=zs)
    assert [v == 0 for v in got] == [g["expect"] for g in groups]


def test_torsion_batches_with_registered_keys(engine, monkeypatch):
    """The same groups with every key registered: the prefilter then takes
    [l]A == O from the key cache's flag (COA_KEY_TORSION_FREE) instead of
    computing it, and must still send the mixed-order groups to the exact
    kernels."""
    monkeypatch.setenv("COA_BATCH_LAT", "1")
    groups = _torsion_groups(seed=6)
    msgs, pks, sigs, offs, zs = _pack(groups)
    try:
        engine.committee_register(pks)
        got = engine.verify_batch_groups(msgs, pks, sigs, offs, zs=zs)
    finally:
        engine.committee_register(np.zeros((0, 32), np.uint8))
    assert [v == 0 for v in got] == [g["expect"] for g in groups]


def test_prefilter_many_groups_agree_with_exact(engine, monkeypatch):
    """C1-like call (300 certificates x 3 votes, under the prefilter's 2,048
    signatures) with corrupt votes, a non-canonical s, an undecodable R and
    an empty group: the prefilter's verdicts equal the exact kernels'."""
    from workloads import key_seeds

    ng, per = 300, 3
    seeds = key_seeds(ng * per)
    msgs = np.frombuffer(b"".join(o.sha512(b"pf" + struct.pack("<Q", g))[:32] for g in range(ng)),
                         np.uint8).reshape(ng, 32).copy()
    pks, sigs = engine.sign_many(seeds, np.repeat(msgs, per, axis=0))
    sizes = [per] * ng
    sizes[7] = 0  # an empty group (Ok): drop its votes
    keep = np.ones(ng * per, bool)
    keep[7 * per:8 * per] = False
    pks, sigs = pks[keep].copy(), sigs[keep].copy()
    offs = np.zeros(ng + 1, np.uint64)
    offs[1:] = np.cumsum(sizes)
    sigs[int(offs[3]) + 1, 40] ^= 8
    sigs[int(offs[100]), 32:] = np.frombuffer((o.L + 2).to_bytes(32, "little"), np.uint8)
    sigs[int(offs[200]) + 2, :32] = np.frombuffer(bytes.fromhex("02" + "00" * 31), np.uint8)
    pks[int(offs[250]) + 1, 5] ^= 1
    got = {}
    for r in ("1", "0"):
        monkeypatch.setenv("COA_BATCH_LAT", r)
        got[r] = engine.verify_batch_groups(msgs, pks, sigs, offs, rng_seed=31)
    assert list(got["1"]) == list(got["0"])
    assert sorted(np.nonzero(got["1"])[0].tolist()) == [3, 100, 200, 250]


def test_committee100_certificates(engine):
    """C3 shape: 67 votes per certificate from a committee of 100."""
    from workloads import key_seeds

    seeds = key_seeds(100)
    pks_all = engine.public_keys(seeds)
    ncert = 24
    msgs = np.frombuffer(b"".join(o.sha512(b"cert" + struct.pack("<Q", c))[:32] for c in range(ncert)),
                         np.uint8).reshape(ncert, 32).copy()
    vseeds, vmsgs = [], []
    for c in range(ncert):
        for j in range(67):
            vseeds.append(seeds[(c + j) % 100])
            vmsgs.append(msgs[c])
    pks, sigs = engine.sign_many(np.array(vseeds), np.array(vmsgs))
    offs = np.arange(0, ncert * 67 + 1, 67, dtype=np.uint64)
    assert (engine.verify_batch_groups(msgs, pks, sigs, offs, rng_seed=7) == 0).all()
    sigs[5 * 67 + 3, 33] ^= 2  # corrupt one vote of certificate 5
    v = engine.verify_batch_groups(msgs, pks, sigs, offs, rng_seed=0)
    assert v[5] == 1 and (np.delete(v, 5) == 0).all()
    assert (pks[:67] == pks_all[np.arange(67) % 100]).all()
