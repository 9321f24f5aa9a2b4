"""CPU: the C restatement of dalek's algorithms (oracle/coa_oracle.c, the
on-box oracle and CPU baseline) agrees with every golden fixture and with the
Python oracle on random adversarial mixes."""
import random
import struct

import numpy as np

import coa_oracle as co
import ed25519_ref as o
from conftest import load_golden


def test_c_oracle_verify_vectors():
    for v in load_golden("verify_vectors.json"):
        got = co.verify_strict(bytes.fromhex(v["msg"]), bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]))
        assert got == v["expect"], (v["class"], v["note"])


def test_c_oracle_batch_vectors():
    for g in load_golden("batch_vectors.json"):
        got = co.verify_batch(bytes.fromhex(g["msg"]), [bytes.fromhex(p) for p in g["pks"]],
                              [bytes.fromhex(s) for s in g["sigs"]], [int(z, 16) for z in g["zs"]])
        assert got == g["expect"], g["name"]


def test_c_oracle_sha512():
    for v in load_golden("sha512_vectors.json"):
        assert co.sha512(bytes.fromhex(v["msg"])).hex() == v["sha512"]


def test_c_oracle_mixed_pool_accepted():
    for v in load_golden("mixed_order_pool.json"):
        assert co.verify_strict(bytes.fromhex(v["msg"]), bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]))


def test_c_vs_python_oracle_random_mix():
    from workloads import adversarial_mix

    n = 160
    seeds = [o.sha512(b"coa-key" + struct.pack("<Q", i))[:32] for i in range(n)]
    ms = [o.sha512(struct.pack("<Q", i))[:32] for i in range(n)]
    pks = np.frombuffer(b"".join(o.public_key(s) for s in seeds), np.uint8).reshape(n, 32).copy()
    sigs = np.frombuffer(b"".join(o.sign(s, m) for s, m in zip(seeds, ms)), np.uint8).reshape(n, 64).copy()
    msgs = np.frombuffer(b"".join(ms), np.uint8).reshape(n, 32).copy()
    pool = [(bytes.fromhex(v["msg"]), bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]))
            for v in load_golden("mixed_order_pool.json")]
    msgs, pks, sigs, cls = adversarial_mix(msgs, pks, sigs, frac=0.5, seed=3, mixed_pool=pool)
    c = co.verify_strict_many(msgs, pks, sigs, 2)
    py = np.array([0 if o.verify_strict(bytes(msgs[i]), bytes(pks[i]), bytes(sigs[i])) else 1 for i in range(n)])
    assert (c == py).all()
    assert set(cls[cls >= 0]) == set(range(8))
    assert (c[cls == 7] == 0).all()        # mixed-order A accepted
    assert (c[(cls >= 0) & (cls < 6)] == 1).all()


def test_c_oracle_batch_random_z_torsion_free():
    rng = random.Random(11)
    m = o.sha512(b"m")[:32]
    seeds = [o.sha512(bytes([i]))[:32] for i in range(5)]
    pks = [o.public_key(s) for s in seeds]
    sigs = [o.sign(s, m) for s in seeds]
    for _ in range(3):
        zs = [rng.getrandbits(128) for _ in seeds]
        assert co.verify_batch(m, pks, sigs, zs) and o.verify_batch(m, pks, sigs, zs)


def test_libsodium_second_reference_agrees_on_canonical_triples():
    """bench.py's second CPU reference (oracle/sodium_drive.c) gives dalek's
    verdicts on canonical valid / tampered triples (the only inputs it is
    timed on); skipped where the image has no libsodium."""
    import pytest

    n = 48
    seeds = [o.sha512(b"sod" + struct.pack("<Q", i))[:32] for i in range(n)]
    ms = [o.sha512(struct.pack("<Q", 7 * i))[:32] for i in range(n)]
    sigs = [bytearray(o.sign(s, m)) for s, m in zip(seeds, ms)]
    ms = [bytearray(m) for m in ms]
    for i in range(0, n, 3):
        (sigs[i] if i % 2 else ms[i])[i % 32] ^= 1 << (i % 8)   # tamper R/s or the message
    A = lambda rows, w: np.frombuffer(b"".join(bytes(r) for r in rows), np.uint8).reshape(n, w).copy()  # noqa
    msgs, pks, sg = A(ms, 32), A([o.public_key(s) for s in seeds], 32), A(sigs, 64)
    got = co.sodium_verify_many(msgs, pks, sg, 2)
    if got is None:
        pytest.skip("libsodium not present")
    assert (got[0] == co.verify_strict_many(msgs, pks, sg, 2)).all()
    assert int(got[0].sum()) == len(range(0, n, 3))
