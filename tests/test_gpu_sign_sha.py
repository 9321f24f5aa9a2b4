"""GPU parity: RFC 8032 signing (Signature::new) and SHA-512 digests
(Sha512::digest at worker/src/processor.rs:38 and the primary digests)."""
import hashlib
import struct

import numpy as np
import pytest

import ed25519_ref as o
from conftest import load_golden

pytestmark = pytest.mark.gpu


def test_sign_matches_oracle(engine):
    seeds = [o.sha512(b"coa-key" + struct.pack("<Q", i))[:32] for i in range(40)]
    msgs = [o.sha512(struct.pack("<Q", i))[:32] for i in range(40)]
    pks, sigs = engine.sign_many(np.frombuffer(b"".join(seeds), np.uint8).reshape(40, 32),
                                 np.frombuffer(b"".join(msgs), np.uint8).reshape(40, 32))
    for i in range(40):
        assert bytes(pks[i]) == o.public_key(seeds[i])
        assert bytes(sigs[i]) == o.sign(seeds[i], msgs[i])
    ref = load_golden("reference_crypto.json")
    s = np.frombuffer(b"".join(bytes.fromhex(x) for x in ref["seeds"]), np.uint8).reshape(4, 32)
    assert [bytes(p).hex() for p in engine.public_keys(s)] == ref["public_keys"]


@pytest.mark.parametrize("msg_len", [0, 1, 17, 64, 100, 200])
def test_sign_variable_length(engine, msg_len):
    rng = np.random.default_rng(msg_len)
    seeds = rng.integers(0, 256, (8, 32), dtype=np.uint8)
    msgs = rng.integers(0, 256, (8, msg_len), dtype=np.uint8)
    pks, sigs = engine.sign_many(seeds, msgs)
    for i in range(8):
        assert bytes(sigs[i]) == o.sign(bytes(seeds[i]), bytes(msgs[i]))


def test_sha512_golden(engine):
    vecs = load_golden("sha512_vectors.json")
    out = engine.sha512_many([bytes.fromhex(v["msg"]) for v in vecs])
    for v, d in zip(vecs, out):
        assert bytes(d).hex() == v["sha512"]


def test_sha512_random_lengths_and_alignment(engine):
    rng = np.random.default_rng(3)
    msgs = [bytes(rng.integers(0, 256, int(ln), dtype=np.uint8)) for ln in rng.integers(0, 2000, 257)]
    out = engine.sha512_many(msgs)
    for m, d in zip(msgs, out):
        assert bytes(d) == hashlib.sha512(m).digest()


def test_reference_batch_digest(engine):
    ref = load_golden("reference_crypto.json")
    d = engine.digest_many([bytes.fromhex(ref["serialized_batch"])])[0]
    assert bytes(d).hex() == ref["batch_digest"]
    assert engine.digest_many([b"Hello, world!"])[0] == engine.Digest(bytes.fromhex(ref["hello_digest"]))


def test_worker_batch_500kb(engine):
    """C4 shape: bincode WorkerMessage::Batch of 977 x 512 B txs (508,052 B)."""
    from workloads import worker_batch

    batches = [worker_batch(b) for b in range(6)]
    assert all(len(b) == 508_052 for b in batches)
    out = engine.sha512_many(batches)
    for b, d in zip(batches, out):
        assert bytes(d) == hashlib.sha512(b).digest()


@pytest.mark.parametrize("lanes", ["1", "2", "4", "8", "16", "32", "64", "auto"])
def test_sha512_lanes_per_message_ragged(engine, lanes, monkeypatch):
    """SHA-512 with L lanes per message (shared message schedule in LDS):
    ragged lengths around the padding boundaries, multi-block, empty and
    mixed lengths inside one wave, vs hashlib."""
    import hashlib
    import random

    if lanes != "auto":
        monkeypatch.setenv("COA_SHA_LANES", lanes)
    rng = random.Random(int(lanes) if lanes != "auto" else 99)
    lens = [0, 1, 111, 112, 113, 127, 128, 129, 239, 240, 255, 256, 1000, 3336, 9001]
    lens += [rng.randrange(0, 5000) for _ in range(70)]
    msgs = [bytes(rng.getrandbits(8) for _ in range(n)) for n in lens]
    got = engine.sha512_many(msgs)
    for m, g in zip(msgs, got):
        assert bytes(g) == hashlib.sha512(m).digest(), len(m)


@pytest.mark.parametrize("lanes", ["2", "4", "8", "64"])
@pytest.mark.parametrize("prefetch", ["0", "1"])
def test_sha512_prefetched_whole_blocks(engine, lanes, prefetch, monkeypatch):
    """k_sha512_ml's prefetched loop over the groups of blocks that are whole
    for every message of a wave, then the padded tail groups: 16-byte-aligned
    messages (lengths multiples of 16, so each starts aligned in the packed
    buffer) of different block counts in one wave -- the wave-uniform end of
    the whole groups falls inside some messages and after others -- plus a
    wave whose last groups have dead lanes; with and without the prefetch
    (COA_SHA_PREFETCH), vs hashlib."""
    import hashlib
    import random

    monkeypatch.setenv("COA_SHA_LANES", lanes)
    monkeypatch.setenv("COA_SHA_PREFETCH", prefetch)
    rng = random.Random(7 + int(lanes))
    lens = [16 * rng.randrange(0, 200) for _ in range(45)] + [128 * 40, 128 * 40 + 112, 16 * 513]
    msgs = [bytes(rng.getrandbits(8) for _ in range(n)) for n in lens]
    got = engine.sha512_many(msgs)
    for m, g in zip(msgs, got):
        assert bytes(g) == hashlib.sha512(m).digest(), len(m)
