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


def test_c_oracle_certificate_verify_many_matches_pieces():
    """coa_oracle_certificate_verify_many (the C3 all-core CPU baseline and
    the C3 parity checker) gives, per certificate, the bits of the three
    single checks it is made of, on any thread count."""
    rnd = random.Random(3)
    seeds = [bytes([i + 1]) * 32 for i in range(5)]
    pks = [o.public_key(s) for s in seeds]
    hin, ids, origins, hsigs, vp, vs, offs, exp = [], [], [], [], [], [], [0], []
    for c in range(6):
        author = c % 5
        h = pks[author] + struct.pack("<Q", 7) + bytes(rnd.getrandbits(8) for _ in range(40))
        hid = o.sha512(h)[:32]
        sig = o.sign(seeds[author], hid)
        cd = o.sha512(hid + struct.pack("<Q", 7) + pks[author])[:32]
        votes = [(pks[v], o.sign(seeds[v], cd)) for v in range(4)]
        bits = 0
        if c == 1:
            h = h[:-1] + bytes([h[-1] ^ 1]); bits |= 1
        if c == 2:
            sig = sig[:40] + bytes([sig[40] ^ 1]) + sig[41:]; bits |= 2
        if c == 3:
            votes[2] = (votes[2][0], votes[2][1][:5] + bytes([votes[2][1][5] ^ 1]) + votes[2][1][6:]); bits |= 4
        if c == 4:
            votes[0] = (pks[4], votes[0][1]); bits |= 4
        hin.append(h); ids.append(hid); origins.append(pks[author]); hsigs.append(sig)
        vp += [p for p, _ in votes]; vs += [s for _, s in votes]; offs.append(offs[-1] + len(votes))
        exp.append(bits)
    n = len(hin)
    zs = np.frombuffer(bytes(rnd.getrandbits(8) for _ in range(16 * len(vp))), np.uint8).reshape(-1, 16)
    arr = lambda xs, w: np.frombuffer(b"".join(xs), np.uint8).reshape(-1, w)  # noqa: E731
    for threads in (1, 3, 8):
        got = co.certificate_verify_many(hin, arr(ids, 32), arr(origins, 32), arr(hsigs, 64), 7, arr(vp, 32),
                                         arr(vs, 64), np.array(offs, np.uint64), zs, threads)
        assert list(got) == exp
    # and each certificate's bits agree with the one-certificate helper's verdict
    for c in range(n):
        lo, hi = offs[c], offs[c + 1]
        ok = co.certificate_verify(hin[c], ids[c], origins[c], hsigs[c], 7, vp[lo:hi], vs[lo:hi],
                                   [int.from_bytes(bytes(z), "little") for z in zs[lo:hi]])
        assert ok == (exp[c] == 0)
