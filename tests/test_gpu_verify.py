"""GPU parity: crypto::Signature::verify (dalek 1.0.1 verify_strict) through
the C ABI vs the oracle-generated golden vectors and the oracle itself."""
import random
import struct

import numpy as np
import pytest

import ed25519_ref as o
from conftest import load_golden

pytestmark = pytest.mark.gpu


def _run(engine, vecs):
    by_len = {}
    for i, v in enumerate(vecs):
        by_len.setdefault(len(v["msg"]) // 2, []).append(i)
    got = [None] * len(vecs)
    for ln, idx in by_len.items():
        msgs = np.array([list(bytes.fromhex(vecs[i]["msg"])) for i in idx], np.uint8).reshape(len(idx), ln)
        pks = np.array([list(bytes.fromhex(vecs[i]["pk"])) for i in idx], np.uint8)
        sigs = np.array([list(bytes.fromhex(vecs[i]["sig"])) for i in idx], np.uint8)
        out = engine.verify_strict_many(msgs, pks, sigs)
        for j, i in enumerate(idx):
            got[i] = out[j] == 0
    return got


def test_golden_verify_vectors(engine):
    vecs = load_golden("verify_vectors.json")
    got = _run(engine, vecs)
    bad = [(v["class"], v["note"]) for v, g in zip(vecs, got) if g != v["expect"]]
    assert not bad, bad


def test_reference_crypto_tests(engine):
    """crypto/src/tests/crypto_tests.rs:49-115 through the mirrored API."""
    ref = load_golden("reference_crypto.json")
    pks = [engine.PublicKey(bytes.fromhex(p)) for p in ref["public_keys"]]
    hello = engine.Digest(bytes.fromhex(ref["hello_digest"]))
    sig = engine.Signature.from_bytes(bytes.fromhex(ref["hello_sig_key3"]))
    sig.verify(hello, pks[3])  # verify_valid_signature
    with pytest.raises(engine.CryptoError):  # verify_invalid_signature
        sig.verify(engine.Digest(bytes.fromhex(ref["bad_digest"])), pks[3])
    votes = [(engine.PublicKey(bytes.fromhex(p)), engine.Signature.from_bytes(bytes.fromhex(s)))
             for p, s in ref["batch_valid"]]
    engine.Signature.verify_batch(hello, votes)  # verify_valid_batch
    votes = [(engine.PublicKey(bytes.fromhex(p)), engine.Signature.from_bytes(bytes.fromhex(s)))
             for p, s in ref["batch_invalid"]]
    with pytest.raises(engine.CryptoError):  # verify_invalid_batch
        engine.Signature.verify_batch(hello, votes)
    # Signature::default() alone
    with pytest.raises(engine.CryptoError):
        engine.Signature().verify(hello, pks[3])


def test_empty_and_single(engine):
    z = np.zeros((0, 32), np.uint8)
    assert engine.verify_strict_many(z, z, np.zeros((0, 64), np.uint8)).shape == (0,)


def _mixed_inputs(n, seed):
    """n oracle-signed items with ~1/4 adversarial mutations; oracle verdicts."""
    rng = random.Random(seed)
    so = o.small_order_encodings()
    msgs, pks, sigs, exp = [], [], [], []
    for i in range(n):
        sd = o.sha512(b"coa-key" + struct.pack("<Q", i % 97))[:32]
        m = o.sha512(struct.pack("<Q", seed * 1000003 + i))[:32]
        pk = o.public_key(sd)
        sg = o.sign(sd, m)
        c = rng.randrange(8)
        if c == 1:
            sg = sg[:32] + (int.from_bytes(sg[32:], "little") + o.L).to_bytes(32, "little")
        elif c == 2:
            b = bytearray(sg); b[rng.randrange(64)] ^= 1 << rng.randrange(8); sg = bytes(b)
        elif c == 3:
            sg = rng.choice(so) + sg[32:]
        elif c == 4:
            pk = rng.choice(so)
        elif c == 5:
            b = bytearray(m); b[rng.randrange(32)] ^= 1; m = bytes(b)
        msgs.append(m); pks.append(pk); sigs.append(sg)
        exp.append(o.verify_strict(m, pk, sg))
    a = lambda xs, w: np.frombuffer(b"".join(xs), np.uint8).reshape(len(xs), w).copy()
    return a(msgs, 32), a(pks, 32), a(sigs, 64), np.array(exp)


def test_random_mixed_vs_oracle(engine):
    msgs, pks, sigs, exp = _mixed_inputs(300, 7)
    got = engine.verify_strict_many(msgs, pks, sigs) == 0
    assert (got == exp).all(), np.nonzero(got != exp)


@pytest.mark.parametrize("n", [300_000, 2_100_000])
def test_grid_stride_large_n_all_valid(engine, n):
    """More items than verify lanes (grid-stride path), and more than one
    split chunk (2^21 items) -- size-independent property: every honestly
    generated signature is accepted, and flipping one bit of s in every 7th
    item is rejected exactly there."""
    rng = np.random.default_rng(1)
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    pks, sigs = engine.sign_many(seeds, msgs)
    bad = np.arange(n) % 7 == 3
    sigs2 = sigs.copy()
    sigs2[bad, 40] ^= 1
    v = engine.verify_strict_many(msgs, pks, sigs2)
    assert (v[~bad] == 0).all()
    assert (v[bad] == 1).all()


def test_wide_comb_table_consistent(engine):
    """Every entry of the 654 MB HBM comb of B is m * 2^(20 j) * B: checked on
    the device against its neighbours, independently of how it was built."""
    assert engine.self_test(0) == 0


def test_wide_comb_matches_radix256_comb(engine, monkeypatch):
    """[e]B through the wide comb (default) and through the radix-256 comb
    (COA_WCOMB=0, read per call) give the same verdicts on valid, tampered
    and adversarial triples."""
    msgs, pks, sigs, exp = _mixed_inputs(400, 11)
    wide = engine.verify_strict_many(msgs, pks, sigs)
    monkeypatch.setenv("COA_WCOMB", "0")
    narrow = engine.verify_strict_many(msgs, pks, sigs)
    assert (wide == narrow).all()
    assert ((wide == 0) == exp).all()
