"""GPU parity: committee key cache (f2) and the fused Certificate::verify
crypto (f3, coa_certificate_verify[_many]) against the oracle.

The expected status bits of every certificate come from the C restatement of
dalek (oracle/coa_oracle.c) and hashlib:
  bit 1  SHA-512(header bytes)[..32] != header.id   (primary/src/messages.rs:49-51)
  bit 2  !verify_strict(header.id, author, sig)     (messages.rs:64-66)
  bit 4  !verify_batch(Certificate::digest, votes)  (messages.rs:214)
Adversarial classes cover cached and uncached keys, small-order / mixed-order
/ off-curve keys in the registered committee, non-canonical s, off-curve R,
R = identity (accepted by verify_batch, rejected by verify_strict), wrong
signers and torsion-perturbed R (whose batch verdict depends on the weights:
checked against verify_batch_groups with the same seed).  Every case runs in
both kernel variants (64 lanes per signature -- latency, 1 -- throughput)
and through the single-certificate entry point."""
import hashlib
import os
import random
import struct

import numpy as np
import pytest

import coa_oracle as co
import ed25519_ref as o
from conftest import load_golden

pytestmark = pytest.mark.gpu

L_ORDER = o.L


def _t8():
    for T in o.torsion_points():
        if not o.is_identity(o.pdbl(o.pdbl(T))):
            return T
    raise AssertionError


def _expected_flags(pk):
    P = o.decompress(pk)
    if P is None:
        return 0
    f = 1
    if o.is_small_order(P):
        f |= 2
    if o.is_identity(o.pmul(L_ORDER, P)):
        f |= 4
    return f


def _engine_order(keys):
    return sorted(set(keys), key=lambda k: struct.unpack("<8I", k))


def _golden_pks(cls, n):
    out = []
    for v in load_golden("verify_vectors.json"):
        if v["class"] == cls and bytes.fromhex(v["pk"]) not in out:
            out.append(bytes.fromhex(v["pk"]))
    return out[:n]


def test_key_flags(engine):
    honest = [bytes(p) for p in engine.public_keys(np.array([list(o.sha512(b"kf" + bytes([i]))[:32])
                                                            for i in range(6)], np.uint8))]
    keys = honest + _golden_pks("small_order_A", 3) + _golden_pks("noncanonical_A", 3) + \
        _golden_pks("off_curve", 2) + _golden_pks("mixed_order_A", 2)
    n = engine.committee_register(np.array([list(k) for k in keys + keys[:2]], np.uint8))  # duplicates collapse
    order = _engine_order(keys)
    assert n == len(order)
    got = engine.committee_key_flags()
    exp = [_expected_flags(k) for k in order]
    assert list(got) == exp
    assert {f for f in exp} >= {0, 1 | 4, 1 | 2, 1}  # off-curve, honest, small order, mixed order


# ---------------------------------------------------------------------------
def _sign(engine, seeds, msgs):
    pks, sigs = engine.sign_many(np.array([list(s) for s in seeds], np.uint8),
                                 np.array([list(m) for m in msgs], np.uint8))
    return [bytes(p) for p in pks], [bytes(s) for s in sigs]


def _cert_digest(hid, rnd, origin):
    return hashlib.sha512(hid + struct.pack("<Q", rnd) + origin).digest()[:32]


class World:
    """A small committee with honest and adversarial members."""

    def __init__(self, engine, n_honest=10):
        self.engine = engine
        self.seeds = [o.sha512(b"coa-key" + struct.pack("<Q", 9000 + i))[:32] for i in range(n_honest)]
        self.pks = [bytes(p) for p in engine.public_keys(np.array([list(s) for s in self.seeds], np.uint8))]
        # mixed-order member: A = aB + T8 (its secret a is known)
        self.T8 = _t8()
        self.mx_seed = o.sha512(b"mixed-member")[:32]
        self.mx_a, _ = o.expand_seed(self.mx_seed)
        self.mx_pk = o.compress(o.padd(o.pmul(self.mx_a, o.B), self.T8))
        # an honest key that is NOT registered
        self.out_seed = o.sha512(b"outsider")[:32]
        self.out_pk = o.public_key(self.out_seed)
        self.registered = self.pks + [self.mx_pk] + _golden_pks("small_order_A", 1) + _golden_pks("off_curve", 1)
        self.T2 = next(T for T in o.torsion_points() if not o.is_identity(T) and o.is_identity(o.pdbl(T)))

    def register(self):
        return self.engine.committee_register(np.array([list(k) for k in self.registered], np.uint8))

    def mixed_sign(self, msg, rng):
        """Signature by the mixed-order member whose R absorbs the torsion so
        the cofactorless per-signature equation holds."""
        while True:
            r = rng.getrandbits(256) % L_ORDER
            for j in range(8):
                R = o.padd(o.pmul(r, o.B), o.pmul(j, self.T8))
                Rb = o.compress(R)
                k = o.scalar_from_hash(o.sha512(Rb + self.mx_pk + msg))
                if (j + k) % 8 == 0:
                    return Rb + ((r + k * self.mx_a) % L_ORDER).to_bytes(32, "little")

    def identity_r_sign(self, seed, msg):
        """R = identity, s = k*a: [s]B - [k]A == R, so verify_batch accepts and
        verify_strict rejects (small-order R)."""
        a, _ = o.expand_seed(seed)
        A = o.compress(o.pmul(a, o.B))
        Rb = o.compress(o.IDENT)
        k = o.scalar_from_hash(o.sha512(Rb + A + msg))
        return Rb + (k * a % L_ORDER).to_bytes(32, "little")

    def certificate(self, c, hdr_len, n_votes, rnd=7):
        rng = random.Random(c)
        hdr = bytes(rng.getrandbits(8) for _ in range(hdr_len))
        hid = hashlib.sha512(hdr).digest()[:32]
        a = c % len(self.seeds)
        _, (hsig,) = _sign(self.engine, [self.seeds[a]], [hid])
        origin = self.pks[a]
        cd = _cert_digest(hid, rnd, origin)
        voters = [(c + j) % len(self.seeds) for j in range(n_votes)]
        vpks, vsigs = _sign(self.engine, [self.seeds[v] for v in voters], [cd] * n_votes)
        return {"hdr": hdr, "id": hid, "origin": origin, "hsig": hsig, "round": rnd, "vpks": vpks,
                "vsigs": vsigs, "voters": voters, "a": a}


def _bump_s(sig, delta):
    s = (int.from_bytes(sig[32:], "little") + delta) % (1 << 256)
    return sig[:32] + s.to_bytes(32, "little")


def _flip(b, i, bit=1):
    x = bytearray(b)
    x[i] ^= bit
    return bytes(x)


def _mutations(w):
    """(name, mutate(cert, rng) -> cert, deterministic?)"""
    so_r = o.small_order_encodings()[3]
    off_r = bytes.fromhex(load_golden("verify_vectors.json")[0]["sig"])[:32]  # replaced below
    for v in load_golden("verify_vectors.json"):
        if v["class"] == "off_curve" and o.decompress(bytes.fromhex(v["sig"])[:32]) is None:
            off_r = bytes.fromhex(v["sig"])[:32]
            break
    assert o.decompress(off_r) is None

    def hdr_byte(c, r):
        c["hdr"] = _flip(c["hdr"], len(c["hdr"]) // 2)
        return c

    def hsig_s(c, r):
        c["hsig"] = _flip(c["hsig"], 40)
        return c

    def hsig_s_plus_l(c, r):
        c["hsig"] = _bump_s(c["hsig"], L_ORDER)
        return c

    def hsig_small_r(c, r):
        c["hsig"] = so_r + c["hsig"][32:]
        return c

    def hsig_identity_r(c, r):
        c["hsig"] = w.identity_r_sign(w.seeds[c["a"]], c["id"])
        return c

    def hdr_mixed_author(c, r):
        c["origin"] = w.mx_pk
        c["hsig"] = w.mixed_sign(c["id"], r)
        cd = _cert_digest(c["id"], c["round"], c["origin"])
        _, c["vsigs"] = _sign(w.engine, [w.seeds[v] for v in c["voters"]], [cd] * len(c["voters"]))
        return c

    def hdr_small_author(c, r):
        c["origin"] = _golden_pks("small_order_A", 1)[0]
        cd = _cert_digest(c["id"], c["round"], c["origin"])
        _, c["vsigs"] = _sign(w.engine, [w.seeds[v] for v in c["voters"]], [cd] * len(c["voters"]))
        return c

    def vote_s(c, r):
        c["vsigs"][1] = _flip(c["vsigs"][1], 33)
        return c

    def vote_s_plus_l(c, r):
        c["vsigs"][2] = _bump_s(c["vsigs"][2], L_ORDER)
        return c

    def vote_off_curve_r(c, r):
        c["vsigs"][0] = off_r + c["vsigs"][0][32:]
        return c

    def vote_wrong_key(c, r):
        c["vpks"][3] = w.pks[(c["voters"][3] + 1) % len(w.pks)]
        return c

    def vote_off_curve_key(c, r):
        c["vpks"][1] = _golden_pks("off_curve", 1)[0]
        return c

    def vote_identity_r(c, r):
        cd = _cert_digest(c["id"], c["round"], c["origin"])
        c["vsigs"][2] = w.identity_r_sign(w.seeds[c["voters"][2]], cd)
        return c

    def vote_outsider(c, r):
        cd = _cert_digest(c["id"], c["round"], c["origin"])
        c["vpks"][0] = w.out_pk
        c["vsigs"][0] = o.sign(w.out_seed, cd)
        return c

    def outsider_bad_vote(c, r):
        c = vote_outsider(c, r)
        c["vsigs"][1] = _flip(c["vsigs"][1], 50)
        return c

    def id_and_votes(c, r):
        return vote_s(hdr_byte(c, r), r)

    def vote_torsion_r(c, r):  # R = rB + T2 hashed as such: E = T2, verdict depends on the weights
        cd = _cert_digest(c["id"], c["round"], c["origin"])
        a, _ = o.expand_seed(w.seeds[c["voters"][1]])
        rr = r.getrandbits(256) % L_ORDER
        Rb = o.compress(o.padd(o.pmul(rr, o.B), w.T2))
        k = o.scalar_from_hash(o.sha512(Rb + c["vpks"][1] + cd))
        c["vsigs"][1] = Rb + ((rr + k * a) % L_ORDER).to_bytes(32, "little")
        return c

    def vote_mixed_member(c, r):  # torsion key: batch verdict depends on the weights
        cd = _cert_digest(c["id"], c["round"], c["origin"])
        c["vpks"][4] = w.mx_pk
        c["vsigs"][4] = w.mixed_sign(cd, r)
        return c

    return [("ok", lambda c, r: c, True), ("hdr_byte", hdr_byte, True), ("hsig_s", hsig_s, True),
            ("hsig_s_plus_l", hsig_s_plus_l, True), ("hsig_small_r", hsig_small_r, True),
            ("hsig_identity_r", hsig_identity_r, True), ("hdr_mixed_author", hdr_mixed_author, True),
            ("hdr_small_author", hdr_small_author, True), ("vote_s", vote_s, True),
            ("vote_s_plus_l", vote_s_plus_l, True), ("vote_off_curve_r", vote_off_curve_r, True),
            ("vote_wrong_key", vote_wrong_key, True), ("vote_off_curve_key", vote_off_curve_key, True),
            ("vote_identity_r", vote_identity_r, True), ("vote_outsider", vote_outsider, True),
            ("outsider_bad_vote", outsider_bad_vote, True), ("id_and_votes", id_and_votes, True),
            ("vote_torsion_r", vote_torsion_r, False), ("vote_mixed_member", vote_mixed_member, False)]


def _oracle_bits(c):
    bits = 0
    if hashlib.sha512(c["hdr"]).digest()[:32] != c["id"]:
        bits |= 1
    if not co.verify_strict(c["id"], c["origin"], c["hsig"]):
        bits |= 2
    cd = _cert_digest(c["id"], c["round"], c["origin"])
    rng = random.Random(7)
    zs = [rng.getrandbits(128) for _ in c["vpks"]]
    if not co.verify_batch(cd, c["vpks"], c["vsigs"], zs):
        bits |= 4
    return bits


def _many(engine, certs, seed=0):
    ids = np.array([list(c["id"]) for c in certs], np.uint8)
    ors = np.array([list(c["origin"]) for c in certs], np.uint8)
    hs = np.array([list(c["hsig"]) for c in certs], np.uint8)
    rounds = np.array([c["round"] for c in certs], np.uint64)
    vp = np.array([list(p) for c in certs for p in c["vpks"]], np.uint8).reshape(-1, 32)
    vs = np.array([list(s) for c in certs for s in c["vsigs"]], np.uint8).reshape(-1, 64)
    offs = np.zeros(len(certs) + 1, np.uint64)
    offs[1:] = np.cumsum([len(c["vpks"]) for c in certs])
    return engine.certificate_verify_many([c["hdr"] for c in certs], ids, ors, hs, rounds, vp, vs, offs,
                                          rng_seed=seed)


def _single(engine, c, seed=0):
    vp = np.array([list(p) for p in c["vpks"]], np.uint8).reshape(-1, 32)
    vs = np.array([list(s) for s in c["vsigs"]], np.uint8).reshape(-1, 64)
    return engine.certificate_verify(c["hdr"], c["id"], c["origin"], c["hsig"], c["round"], vp, vs, rng_seed=seed)


@pytest.fixture(scope="module")
def world(engine):
    return World(engine)


@pytest.fixture(params=["64", "64/staged", "1/T0", "1/T256", "1/T512", "1/T0/narrow", "1/T0/kw16"])
def lanes(request):
    """Latency kernel (64) and throughput kernel with one signature per lane
    (T0 = default grid) or a grid of 256 / 512 lanes, so each lane shares one
    inversion among several signatures (P compared with R's encoding).
    `narrow`: [s]B and [k](-A) from the radix-256 combs instead of the wide
    HBM comb of B and the keys' wide combs.  `kw16`: the keys' radix-2^16
    wide combs (48 MiB per key) instead of the default radix-2^20 ones (654 MB
    per key; COA_KEY_WCOMB20_MB=0 at registration).  `staged`: one-certificate calls
    through the pinned staging copy instead of the kernel arguments
    (COA_CERT_INLINE=0; certificates over 2,816 bytes take it anyway)."""
    parts = request.param.split("/")
    os.environ["COA_CERT_LANES"] = parts[0]
    if "staged" in parts:
        os.environ["COA_CERT_INLINE"] = "0"
    if len(parts) > 1 and parts[1] != "T0":
        os.environ["COA_CERT_LANES_TOTAL"] = parts[1][1:]
    if "narrow" in parts:
        os.environ["COA_WCOMB"] = "0"
        os.environ["COA_KEY_WCOMB"] = "0"
    if "kw16" in parts:
        os.environ["COA_KEY_WCOMB20_MB"] = "0"
    yield int(parts[0])
    del os.environ["COA_CERT_LANES"]
    os.environ.pop("COA_CERT_INLINE", None)
    os.environ.pop("COA_CERT_LANES_TOTAL", None)
    os.environ.pop("COA_WCOMB", None)
    os.environ.pop("COA_KEY_WCOMB", None)
    os.environ.pop("COA_KEY_WCOMB20_MB", None)


def test_fused_certificates_adversarial(engine, world, lanes):
    world.register()
    muts = [m for m in _mutations(world) if m[2]]
    certs, exp, names = [], [], []
    for i, (name, f, _) in enumerate(muts):
        for rep in range(2):
            c = world.certificate(100 * i + rep, hdr_len=[72, 111, 112, 128, 1000, 3336][(i + rep) % 6],
                                  n_votes=7)
            c = f(c, random.Random(i * 7 + rep))
            certs.append(c)
            exp.append(_oracle_bits(c))
            names.append(name)
    got = _many(engine, certs, seed=77)
    bad = [(n, int(g), e) for n, g, e in zip(names, got, exp) if int(g) != e]
    assert not bad, bad
    # classes are not vacuous
    assert {e for e in exp} >= {0, 1, 2, 4, 5}
    # the single-certificate (latency) entry point agrees
    for c, e in zip(certs[::3], exp[::3]):
        assert _single(engine, c, seed=5) == e


def test_fused_weight_dependent_classes(engine, world, lanes):
    """Torsion-perturbed R and mixed-order voters: dalek's verdict depends on
    its random weights.  The fused path must hand these to the exact RLC
    kernels, so its verdict equals verify_batch_groups' with the same seed
    (one certificate per call: same group index, same weights)."""
    world.register()
    muts = [m for m in _mutations(world) if not m[2]]
    seen = set()
    for i, (name, f, _) in enumerate(muts):
        for rep in range(6):
            c = f(world.certificate(5000 + 10 * i + rep, hdr_len=200, n_votes=7), random.Random(rep))
            cd = _cert_digest(c["id"], c["round"], c["origin"])
            vp = np.array([list(p) for p in c["vpks"]], np.uint8)
            vs = np.array([list(s) for s in c["vsigs"]], np.uint8)
            for seed in (11 + rep, 1000 + rep):
                ref = engine.verify_batch_groups(np.array([list(cd)], np.uint8), vp, vs,
                                                 np.array([0, len(vp)], np.uint64), rng_seed=seed)[0]
                got = _single(engine, c, seed=seed)
                assert got == (4 if ref else 0), (name, rep, seed)
                seen.add(bool(ref))
    assert seen == {True, False}  # both verdicts occur


def test_c3_fused_matches_stepwise(engine, lanes):
    import certificates as C

    committee, batch = C.synth_certificates(24, committee_size=100, n_payload=32, seed=11)
    committee.register()
    assert (C.verify_certificate_batch(batch, committee, rng_seed=3) == 0).all()
    batch.vote_sigs[5 * 67 + 9, 40] ^= 4
    batch.header_sigs[7, 3] ^= 1
    hi = bytearray(batch.header_inputs[9])
    hi[100] ^= 1
    batch.header_inputs[9] = bytes(hi)
    a = C.verify_certificate_batch(batch, committee, rng_seed=3)
    b = C.verify_certificate_batch_stepwise(batch, committee, rng_seed=3)
    assert list(np.nonzero(a)[0]) == [5, 7, 9] and (a == b).all()
    for i in (0, 5, 7, 9):  # object path raises exactly where the stepwise path does
        cert = batch.certificate(i)
        e1 = e2 = None
        try:
            cert.verify(committee)
        except C.DagError as e:
            e1 = type(e).__name__
        try:
            cert.verify_stepwise(committee)
        except C.DagError as e:
            e2 = type(e).__name__
        assert e1 == e2


def test_unregistered_committee_still_exact(engine):
    """Verdict-neutrality of the cache: with an empty committee every
    certificate takes the uncached kernels and the verdicts are unchanged."""
    import certificates as C

    committee, batch = C.synth_certificates(6, committee_size=4, n_payload=2, seed=4)
    batch.vote_sigs[4, 50] ^= 1
    engine.committee_register(np.zeros((0, 32), np.uint8))
    a = C.verify_certificate_batch(batch, committee, rng_seed=1)
    committee.register()
    b = C.verify_certificate_batch(batch, committee, rng_seed=1)
    assert (a == b).all() and list(np.nonzero(a)[0]) == [1]
