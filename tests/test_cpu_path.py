"""CPU: the engine's own CPU path (csrc/coa_cpu.cpp, the coa_cpu_* entries of
include/coa_verify.h) gives the same verdicts as the oracle and the golden
fixtures.  It is what the Rust binding answers with when every GPU context
failed (rust/crypto/src/degrade.rs, COA_ON_ENGINE_FAILURE=cpu); it is never
called implicitly, and none of the GPU parity tests goes through it.

Pinned by: tests/golden/verify_vectors.json (RFC 8032 + adversarial
classes), batch_vectors.json (verify_batch with explicit weights),
sha512_vectors.json, reference_crypto.json (the reference's own crypto tests
recomputed), and a 4,096-item adversarial mix and a certificate round with
injected failures against the C oracle."""
import numpy as np
import pytest

import coa_oracle as co
import ed25519_ref as o
from conftest import load_golden

SEEDS_UNIQUE = 512


@pytest.fixture(scope="module")
def cc():
    import build

    build.build()
    import coa_crypto

    return coa_crypto


def _h(x):
    return bytes.fromhex(x)


def _z(x):  # a batch weight: "0x..." integer -> 16 little-endian bytes
    return int(x, 16).to_bytes(16, "little")


def test_verify_vectors_single(cc):
    L = cc.lib()
    for v in load_golden("verify_vectors.json"):
        m, pk, sig = _h(v["msg"]), _h(v["pk"]), _h(v["sig"])
        rc = L.coa_cpu_ed25519_verify_strict(m, len(m), pk, sig)
        assert rc in (0, 1)
        assert (rc == 0) == v["expect"], (v["class"], v.get("note"))


def test_verify_vectors_many_threads(cc):
    vecs = [v for v in load_golden("verify_vectors.json") if len(v["msg"]) == 64]
    msgs = np.array([list(_h(v["msg"])) for v in vecs], np.uint8)
    pks = np.array([list(_h(v["pk"])) for v in vecs], np.uint8)
    sigs = np.array([list(_h(v["sig"])) for v in vecs], np.uint8)
    for t in (1, 3, 0):
        got = cc.cpu_verify_strict_many(msgs, pks, sigs, nthreads=t)
        assert [bool(x == 0) for x in got] == [v["expect"] for v in vecs]


def test_batch_vectors(cc):
    vecs = load_golden("batch_vectors.json")
    for v in vecs:
        n = len(v["pks"])
        pks = np.array([list(_h(x)) for x in v["pks"]], np.uint8).reshape(n, 32)
        sigs = np.array([list(_h(x)) for x in v["sigs"]], np.uint8).reshape(n, 64)
        zs = np.array([list(_z(x)) for x in v["zs"]], np.uint8).reshape(n, 16)
        msg = np.frombuffer(_h(v["msg"]), np.uint8).reshape(1, 32)
        got = cc.cpu_verify_batch_groups(msg, pks, sigs, [0, n], zs, nthreads=1)
        assert bool(got[0] == 0) == v["expect"], v["name"]
    # all groups in one call, several threads
    msgs = np.array([list(_h(v["msg"])) for v in vecs], np.uint8)
    off = np.cumsum([0] + [len(v["pks"]) for v in vecs]).astype(np.uint64)
    cat = lambda key, w, f=_h: np.array([list(f(x)) for v in vecs for x in v[key]], np.uint8).reshape(-1, w)  # noqa
    got = cc.cpu_verify_batch_groups(msgs, cat("pks", 32), cat("sigs", 64), off, cat("zs", 16, _z), nthreads=4)
    assert [bool(g == 0) for g in got] == [v["expect"] for v in vecs]


def test_verify_batch_random_weights(cc):
    """rng_seed = 0 (OS entropy, dalek's behaviour) and a fixed seed: a valid
    batch is Ok, one corrupted signature makes it Err."""
    seeds = [_h(s) for s in load_golden("reference_crypto.json")["seeds"]]
    msg = bytes(range(32))
    pks = np.array([list(o.public_key(s)) for s in seeds[:6]], np.uint8)
    sigs = np.array([list(o.sign(s, msg)) for s in seeds[:6]], np.uint8)
    L = cc.lib()
    for seed in (0, 7):
        assert L.coa_cpu_ed25519_verify_batch(msg, cc._u8p(pks), cc._u8p(sigs), len(pks), seed) == 0
        bad = sigs.copy()
        bad[3, 40] ^= 1
        assert L.coa_cpu_ed25519_verify_batch(msg, cc._u8p(pks), cc._u8p(bad), len(pks), seed) == 1
    assert L.coa_cpu_ed25519_verify_batch(msg, None, None, 0, 0) == 0  # empty batch: Ok, as dalek


def test_sha512_vectors(cc):
    vecs = load_golden("sha512_vectors.json")
    got = cc.cpu_sha512_many([_h(v["msg"]) for v in vecs], nthreads=2)
    for v, g in zip(vecs, got):
        assert bytes(g).hex() == v["sha512"]


def test_sha512_block_boundaries(cc):
    import hashlib

    msgs = [bytes((i * 7 + j) & 255 for j in range(n)) for i, n in
            enumerate([0, 1, 111, 112, 113, 127, 128, 129, 239, 240, 255, 256, 257, 1000, 508_052])]
    got = cc.cpu_sha512_many(msgs)
    for m, g in zip(msgs, got):
        assert bytes(g) == hashlib.sha512(m).digest()


def test_reference_crypto_fixtures(cc):
    """crypto/src/tests/crypto_tests.rs:26-115 and worker/src/tests/common.rs
    recomputed (tests/golden/reference_crypto.json): the 'Hello, world!'
    digest, verify_valid_signature / verify_invalid_signature,
    verify_valid_batch / verify_invalid_batch (with the fixture's weights)
    and the worker's batch digest."""
    ref = load_golden("reference_crypto.json")
    hello = _h(ref["hello_digest"])
    assert bytes(cc.cpu_sha512_many([b"Hello, world!"])[0][:32]) == hello
    pks = [_h(p) for p in ref["public_keys"]]
    sig = _h(ref["hello_sig_key3"])
    L = cc.lib()
    assert L.coa_cpu_ed25519_verify_strict(hello, 32, pks[3], sig) == 0
    assert L.coa_cpu_ed25519_verify_strict(_h(ref["bad_digest"]), 32, pks[3], sig) == 1
    zs = np.array([list(int(z, 16).to_bytes(16, "little")) for z in ref["batch_zs"]], np.uint8)
    for key, expect in (("batch_valid", 0), ("batch_invalid", 1)):
        votes = ref[key]
        vp = np.array([list(_h(p)) for p, _ in votes], np.uint8)
        vs = np.array([list(_h(x)) for _, x in votes], np.uint8)
        got = cc.cpu_verify_batch_groups(np.frombuffer(hello, np.uint8).reshape(1, 32), vp, vs, [0, len(votes)],
                                         zs[:len(votes)])
        assert got[0] == expect, key
    ser = _h(ref["serialized_batch"])
    assert bytes(cc.cpu_sha512_many([ser])[0][:32]).hex() == ref["batch_digest"]


@pytest.fixture(scope="module")
def mix():
    """4,096 triples: 512 signed on the CPU by the Python oracle, tiled, then
    25 % mutated over the 8 adversarial classes (workloads.adversarial_mix)."""
    from workloads import adversarial_mix, key_seeds, messages

    seeds, msgs = key_seeds(SEEDS_UNIQUE), messages(SEEDS_UNIQUE)
    pks = np.array([list(o.public_key(bytes(s))) for s in seeds], np.uint8)
    sigs = np.array([list(o.sign(bytes(s), bytes(m))) for s, m in zip(seeds, msgs)], np.uint8)
    rep = 4096 // SEEDS_UNIQUE
    pool = [(_h(v["msg"]), _h(v["pk"]), _h(v["sig"])) for v in load_golden("mixed_order_pool.json")]
    return adversarial_mix(np.tile(msgs, (rep, 1)), np.tile(pks, (rep, 1)), np.tile(sigs, (rep, 1)), frac=0.25,
                           seed=0xC0A6, mixed_pool=pool)


def test_adversarial_mix_matches_oracle(cc, mix):
    msgs, pks, sigs, cls = mix
    got = cc.cpu_verify_strict_many(msgs, pks, sigs, nthreads=8)
    exp = co.verify_strict_many(msgs, pks, sigs, 8)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, [(int(i), int(cls[i])) for i in bad[:20]]
    assert set(np.unique(cls[cls >= 0])) == set(range(8))
    assert (got[cls == -1] == 0).all() and (got[cls == 7] == 0).all()
    assert (got[(cls >= 0) & (cls <= 5)] == 1).all()


def test_adversarial_batches_match_oracle(cc):
    """verify_batch over 16 groups of 8 votes, each group signing its own
    digest, a quarter of the votes mutated over the adversarial classes (s
    non-canonical, y >= p, small-order R / A, off-curve, bit flips, mixed
    order): group verdicts equal the oracle's under the same weights."""
    from workloads import adversarial_mix, key_seeds, messages

    g, ng = 8, 16
    n = g * ng
    seeds, digests = key_seeds(n, start=3000), messages(ng, start=3000)
    msgs = np.repeat(digests, g, axis=0)
    pks = np.array([list(o.public_key(bytes(s))) for s in seeds], np.uint8)
    sigs = np.array([list(o.sign(bytes(s), bytes(m))) for s, m in zip(seeds, msgs)], np.uint8)
    pool = [(_h(v["msg"]), _h(v["pk"]), _h(v["sig"])) for v in load_golden("mixed_order_pool.json")]
    _, pks, sigs, cls = adversarial_mix(msgs, pks, sigs, frac=0.25, seed=12, mixed_pool=pool)
    zs = np.random.default_rng(5).integers(0, 256, (n, 16), dtype=np.uint8)
    off = np.arange(0, n + 1, g, dtype=np.uint64)
    got = cc.cpu_verify_batch_groups(digests, pks, sigs, off, zs, nthreads=4)
    zi = [int.from_bytes(bytes(z), "little") for z in zs]
    exp = np.array([0 if co.verify_batch(bytes(digests[k]), pks[k * g:(k + 1) * g], sigs[k * g:(k + 1) * g],
                                         zi[k * g:(k + 1) * g]) else 1 for k in range(ng)], np.uint8)
    assert list(got) == list(exp)
    assert 0 < int(exp.sum()) < ng
    clean = [k for k in range(ng) if (cls[k * g:(k + 1) * g] == -1).all()]
    assert all(got[k] == 0 for k in clean)


def test_certificates_match_oracle(cc):
    """A committee-4 round of 24 certificates (3 votes each) signed on the CPU,
    with header-id, header-signature and vote corruptions injected; the CPU
    path's COA_CERT_* bits equal the oracle's under the same weights."""
    import hashlib

    from workloads import key_seeds

    seeds = key_seeds(4, start=900)
    pks = [o.public_key(bytes(s)) for s in seeds]
    n, q, rnd = 24, 3, 7
    hdrs, ids, origins, hsigs, vpk, vsig = [], [], [], [], [], []
    for c in range(n):
        a = c % 4
        h = bytes([c]) * 40 + pks[a]
        hid = hashlib.sha512(h).digest()[:32]
        hdrs.append(h)
        ids.append(list(hid))
        origins.append(list(pks[a]))
        hsigs.append(list(o.sign(bytes(seeds[a]), hid)))
        cd = hashlib.sha512(hid + rnd.to_bytes(8, "little") + pks[a]).digest()[:32]
        for v in range(q):
            w = (a + 1 + v) % 4
            vpk.append(list(pks[w]))
            vsig.append(list(o.sign(bytes(seeds[w]), cd)))
    ids, origins, hsigs, vpk, vsig = (np.array(x, np.uint8) for x in (ids, origins, hsigs, vpk, vsig))
    hdrs[1] = hdrs[1][:-1] + bytes([hdrs[1][-1] ^ 1])  # header bytes != id
    hsigs[2, 5] ^= 1                                    # header signature
    vsig[3 * 3 + 1, 50] ^= 1                            # one vote
    vpk[3 * 5 + 2] = vpk[3 * 5 + 1]                     # a vote under another key
    origins[6, 3] ^= 4                                  # origin: header sig + digest
    voff = np.arange(0, 3 * n + 1, 3, dtype=np.uint64)
    zs = np.random.default_rng(11).integers(0, 256, (3 * n, 16), dtype=np.uint8)
    rounds = np.full(n, rnd, np.uint64)
    got = cc.cpu_certificate_verify_many(hdrs, ids, origins, hsigs, rounds, vpk, vsig, voff, zs=zs, nthreads=3)
    exp = co.certificate_verify_many(hdrs, ids, origins, hsigs, rounds, vpk, vsig, voff, zs, 2)
    assert list(got) == list(exp)
    assert got[0] == 0 and got[1] == 1 and got[2] == 2 and got[3] == 4 and got[5] == 4 and got[6] & 2
    # fresh weights (rng_seed 0): the same bits on these inputs
    got2 = cc.cpu_certificate_verify_many(hdrs, ids, origins, hsigs, rounds, vpk, vsig, voff)
    assert list(got2) == list(exp)


def test_invalid_arguments(cc):
    L = cc.lib()
    assert L.coa_cpu_ed25519_verify_strict(None, 32, None, None) == -1
    assert L.coa_cpu_ed25519_verify_strict_many(None, 32, None, None, 4, None, 1) == -1
    assert L.coa_cpu_ed25519_verify_strict_many(None, 32, None, None, 0, None, 1) == 0
