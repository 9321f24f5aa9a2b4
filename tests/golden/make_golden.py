"""Generate the committed golden fixtures under tests/golden/ (run in the build
container; the GPU box only reads the JSON).

Sources of truth, in order:
  * the reference's own test fixtures, recomputed: `keys()` =
    StdRng::from_seed([0;32]) (rand 0.7 StdRng = ChaCha20, rand_chacha 0.2) ->
    4 x dalek Keypair::generate (crypto/src/tests/crypto_tests.rs:26-29), the
    "Hello, world!" digest and sign/verify round trips (:49-115), and the
    worker `batch_digest()` over `serialized_batch()`
    (worker/src/tests/common.rs:96-109);
  * RFC 8032 section 7.1 known answers (TEST 1-3);
  * oracle/ed25519_ref.py (dalek 1.0.1 semantics) for every vector, each one
    cross-checked against libsodium 1.0.18 `crypto_sign_verify_detached`
    (present in the build container only) -- the two must agree on every
    vector written here (see SURVEY.md section 8(c) for why they coincide on
    constructible inputs).

Usage: python tests/golden/make_golden.py   (writes *.json next to itself)
"""
import ctypes
import hashlib
import json
import os
import random
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import ed25519_ref as o  # noqa: E402

# ----------------------------------------------------------------- ChaCha20
def _rotl(x, n):
    return ((x << n) | (x >> (32 - n))) & 0xFFFFFFFF


def _qr(s, a, b, c, d):
    s[a] = (s[a] + s[b]) & 0xFFFFFFFF; s[d] = _rotl(s[d] ^ s[a], 16)
    s[c] = (s[c] + s[d]) & 0xFFFFFFFF; s[b] = _rotl(s[b] ^ s[c], 12)
    s[a] = (s[a] + s[b]) & 0xFFFFFFFF; s[d] = _rotl(s[d] ^ s[a], 8)
    s[c] = (s[c] + s[d]) & 0xFFFFFFFF; s[b] = _rotl(s[b] ^ s[c], 7)


def chacha20_keystream(key, nblocks):
    out = b""
    for ctr in range(nblocks):
        st = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574]
        st += list(struct.unpack("<8I", key)) + [ctr, 0, 0, 0]
        w = st[:]
        for _ in range(10):
            _qr(w, 0, 4, 8, 12); _qr(w, 1, 5, 9, 13); _qr(w, 2, 6, 10, 14); _qr(w, 3, 7, 11, 15)
            _qr(w, 0, 5, 10, 15); _qr(w, 1, 6, 11, 12); _qr(w, 2, 7, 8, 13); _qr(w, 3, 4, 9, 14)
        out += struct.pack("<16I", *[(a + b) & 0xFFFFFFFF for a, b in zip(w, st)])
    return out


# ---------------------------------------------------------------- libsodium
_SODIUM = None


def sodium():
    global _SODIUM
    if _SODIUM is None:
        lib = ctypes.CDLL("/opt/conda/lib/libsodium.so")
        assert lib.sodium_init() >= 0
        _SODIUM = lib
    return _SODIUM


def sodium_verify(msg, pk, sig):
    return sodium().crypto_sign_verify_detached(bytes(sig), bytes(msg), ctypes.c_ulonglong(len(msg)), bytes(pk)) == 0


def sodium_sign(seed, msg):
    lib = sodium()
    pk = ctypes.create_string_buffer(32)
    sk = ctypes.create_string_buffer(64)
    lib.crypto_sign_seed_keypair(pk, sk, bytes(seed))
    sig = ctypes.create_string_buffer(64)
    lib.crypto_sign_detached(sig, None, bytes(msg), ctypes.c_ulonglong(len(msg)), sk)
    return pk.raw, sig.raw


# -------------------------------------------------------------- helpers
def H(b):
    return hashlib.sha512(b).digest()


def reference_fixtures():
    ks = chacha20_keystream(bytes(32), 2)
    seeds = [ks[32 * i: 32 * i + 32] for i in range(4)]
    pks = [o.public_key(s) for s in seeds]
    for s, pk in zip(seeds, pks):
        assert sodium_sign(s, b"")[0] == pk
    hello = o.digest32(b"Hello, world!")
    bad = o.digest32(b"Bad message!")
    sig3 = o.sign(seeds[3], hello)
    assert sodium_sign(seeds[3], hello)[1] == sig3
    batch_valid = [(pks[i], o.sign(seeds[i], hello)) for i in (3, 2, 1)]
    batch_invalid = [(pks[i], o.sign(seeds[i], hello)) for i in (3, 2)] + [(pks[1], bytes(64))]
    # worker/src/tests/common.rs:86-100: WorkerMessage::Batch(vec![vec![0;100]; 2]) bincode
    serialized = struct.pack("<IQ", 0, 2) + (struct.pack("<Q", 100) + bytes(100)) * 2
    assert len(serialized) == 228
    zs = [0x1234_5678_9ABC_DEF0_0FED_CBA9_8765_4321 + i for i in range(3)]
    out = {
        "source": "reference tests recomputed: crypto/src/tests/crypto_tests.rs:26-115, worker/src/tests/common.rs:96-109",
        "seeds": [s.hex() for s in seeds],
        "public_keys": [p.hex() for p in pks],
        "hello_digest": hello.hex(),
        "bad_digest": bad.hex(),
        "hello_sig_key3": sig3.hex(),
        "verify_valid_signature": o.verify_strict(hello, pks[3], sig3),
        "verify_invalid_signature": o.verify_strict(bad, pks[3], sig3),
        "batch_valid": [[p.hex(), s.hex()] for p, s in batch_valid],
        "batch_invalid": [[p.hex(), s.hex()] for p, s in batch_invalid],
        "batch_zs": [hex(z) for z in zs],
        "verify_valid_batch": o.verify_batch(hello, [p for p, _ in batch_valid], [s for _, s in batch_valid], zs),
        "verify_invalid_batch": o.verify_batch(hello, [p for p, _ in batch_invalid], [s for _, s in batch_invalid], zs),
        "serialized_batch": serialized.hex(),
        "batch_digest": o.digest32(serialized).hex(),
    }
    assert out["verify_valid_signature"] and not out["verify_invalid_signature"]
    assert out["verify_valid_batch"] and not out["verify_invalid_batch"]
    assert out["batch_digest"] == "24d00f74a0767e74808c8546630902972853fa200e079e582b8b7bdecd7331d8"
    assert out["hello_digest"] == "c1527cd893c124773d811911970c8fe6e857d6df5dc9226bd8a160614c0cd963"
    return out


RFC8032 = [  # RFC 8032 section 7.1 TEST 1, 2, 3 (secret, public, message, signature)
    ("9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60",
     "d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a", "",
     "e5564300c360ac729086e2cc806e828a84877f1eb8e5d974d873e065224901555fb8821590a33bacc61e39701cf9b46bd25bf5f0595bbe24655141438e7a100b"),
    ("4ccd089b28ff96da9db6c346ec114e0f5b8a319f35aba624da8cf6ed4fb8a6fb",
     "3d4017c3e843895a92b70aa74d1b7ebc9c982ccf2ec4968cc0cd55f12af4660c", "72",
     "92a009a9f0d4cab8720e820b5f642540a2b27b5416503f8fb3762223ebdb69da085ac1e43e15996e458f3613d0f11d8c387b2eaeb4302aeeb00d291612bb0c00"),
    ("c5aa8df43f9f837bedb7442f31dcb7b166d38535076f094b85ce3a2e0b4458f7",
     "fc51cd8e6218a1a38da47ed00230f0580816ed13ba3303ac5deb911548908025", "af82",
     "6291d657deec24024827e69c3abe01a30ce548a284743a445e3680d7db5ac3ac18ff9b538d16f290ae67f760984dc6594a7c15e9716ed28dc027beceea1ec40a"),
]


def torsion_gen():
    """An order-8 point T8."""
    for T in o.torsion_points():
        if not o.is_identity(o.pdbl(o.pdbl(T))):
            return T
    raise AssertionError


def mixed_order_signature(seed, msg, T8, rng):
    """A = aB + T8 (mixed order); find R = rB + [j]T8 with j == -k mod 8 so
    the cofactorless equation holds.  dalek verify_strict ACCEPTS these."""
    a, prefix = o.expand_seed(seed)
    A = o.padd(o.pmul(a, o.B), T8)
    Ab = o.compress(A)
    while True:
        r = rng.getrandbits(256) % o.L
        rB = o.pmul(r, o.B)
        for j in range(8):
            R = o.padd(rB, o.pmul(j, T8))
            Rb = o.compress(R)
            k = o.scalar_from_hash(H(Rb + Ab + msg))
            if (j + k) % 8 == 0:
                s = (r + k * a) % o.L
                return Ab, Rb + s.to_bytes(32, "little")


def verify_vectors():
    rng = random.Random(0xC0A5)
    vecs = []

    def add(cls, msg, pk, sig, note=""):
        exp = o.verify_strict(msg, pk, sig)
        lib = sodium_verify(msg, pk, sig)
        assert exp == lib, (cls, note, msg.hex(), pk.hex(), sig.hex(), exp, lib)
        vecs.append({"class": cls, "msg": msg.hex(), "pk": pk.hex(), "sig": sig.hex(), "expect": exp, "note": note})

    for sk, pk, m, sg in RFC8032:
        add("rfc8032", bytes.fromhex(m), bytes.fromhex(pk), bytes.fromhex(sg), "RFC 8032 7.1")
        assert vecs[-1]["expect"]

    seeds = [H(b"coa-key" + struct.pack("<Q", i))[:32] for i in range(64)]
    pks = [o.public_key(s) for s in seeds]
    msgs = [H(struct.pack("<Q", i))[:32] for i in range(64)]
    sigs = [o.sign(s, m) for s, m in zip(seeds, msgs)]
    for i in range(32):
        add("valid", msgs[i], pks[i], sigs[i])
    # other message lengths (multi-block SHA-512 on the k = H(R||A||M) path)
    for ln in (0, 1, 31, 33, 48, 49, 63, 64, 65, 111, 112, 127, 128, 200, 300):
        m = bytes(rng.getrandbits(8) for _ in range(ln))
        add("valid_len", m, pks[ln % 64], o.sign(seeds[ln % 64], m), f"msg_len={ln}")
    so = o.small_order_encodings()
    T8 = torsion_gen()
    for i in range(8):
        m, pk, sg = msgs[i], pks[i], sigs[i]
        s = int.from_bytes(sg[32:], "little")
        # 1. s + l (non-canonical S)
        add("s_plus_l", m, pk, sg[:32] + (s + o.L).to_bytes(32, "little"))
        # 2. s with a high bit set
        b = bytearray(sg); b[63] |= (0x80, 0x40, 0x20, 0x10)[i % 4]
        add("s_high_bit", m, pk, bytes(b), f"bit {(255, 254, 253, 252)[i % 4]}")
        # 6. R or A not on the curve
        while True:
            y = rng.getrandbits(255)
            enc = y.to_bytes(32, "little")
            if o.decompress(enc) is None:
                break
        if i % 2:
            add("off_curve", m, pk, enc + sg[32:], "R off curve")
        else:
            add("off_curve", m, enc, sg, "A off curve")
        # 7. flipped bit in M, R or s
        which = i % 3
        if which == 0:
            mm = bytearray(m); mm[rng.randrange(32)] ^= 1 << rng.randrange(8)
            add("bitflip", bytes(mm), pk, sg, "M")
        elif which == 1:
            b = bytearray(sg); b[rng.randrange(31)] ^= 1 << rng.randrange(8)
            add("bitflip", m, pk, bytes(b), "R")
        else:
            b = bytearray(sg); b[32 + rng.randrange(31)] ^= 1 << rng.randrange(8)
            add("bitflip", m, pk, bytes(b), "s")
        # 8. mixed-order A with torsion-matched R: ACCEPTED (cofactorless)
        Ab, sg8 = mixed_order_signature(seeds[i], m, T8, rng)
        add("mixed_order_A", m, Ab, sg8)
        assert vecs[-1]["expect"], "mixed-order A must be accepted"
        # mixed-order A, R not torsion-matched -> reject
        Rb_bad = o.compress(o.padd(o.decompress(sg8[:32]), T8))
        add("mixed_order_A_unmatched", m, Ab, Rb_bad + sg8[32:])
    # 4./5. small-order R and A, every encoding incl. y>=p and negative zero
    for j, enc in enumerate(so):
        m, pk, sg = msgs[j % 64], pks[j % 64], sigs[j % 64]
        add("small_order_R", m, pk, enc + sg[32:])
        add("small_order_A", m, enc, sg)
        # equation-satisfying small-order A: R = identity, s = 0, k*A == O needs k*A=O;
        # with A of order 1/2 choose msg so that k is even -> cofactorless equation holds
        Apt = o.decompress(enc)
        for t in range(256):
            mm = H(b"so-eq" + bytes([j, t]))[:32]
            Rb = bytes([1]) + bytes(31)
            k = o.scalar_from_hash(H(Rb + enc + mm))
            if o.is_identity(o.pmul(k, Apt)):
                add("small_order_A_eq", mm, enc, Rb + bytes(32), "[0]B - [k]A == R == O")
                break
    # 3. R with y >= p encodings (non-canonical, y-p in [0,18])
    for yy in range(0, 19):
        enc = (yy + o.P).to_bytes(32, "little")
        if yy + o.P >= 1 << 255:
            continue
        for sgn in (0, 1):
            e = bytearray(enc); e[31] |= sgn << 7
            m, pk, sg = msgs[yy], pks[yy], sigs[yy]
            add("noncanonical_R", m, pk, bytes(e) + sg[32:], f"y=p+{yy} sign={sgn}")
            add("noncanonical_A", m, bytes(e), sg, f"y=p+{yy} sign={sgn}")
    # the all-zero Signature::default() (crypto_tests.rs:111)
    add("default_sig", msgs[0], pks[0], bytes(64))
    return vecs


def batch_vectors():
    """Groups for verify_batch with explicit z weights.  Expected verdicts are
    deterministic for these inputs (no torsion component survives the sum), so
    they are z-independent; the torsion-dependent case is documented in
    tests/test_parity_batch.py."""
    rng = random.Random(0xBA7C)
    seeds = [H(b"coa-key" + struct.pack("<Q", i))[:32] for i in range(100)]
    pks = [o.public_key(s) for s in seeds]
    groups = []

    def add(name, msg, items, expect=None):
        zs = [rng.getrandbits(128) for _ in items]
        got = o.verify_batch(msg, [p for p, _ in items], [s for _, s in items], zs)
        if expect is not None:
            assert got == expect, name
        groups.append({"name": name, "msg": msg.hex(), "pks": [p.hex() for p, _ in items],
                       "sigs": [s.hex() for _, s in items], "zs": [hex(z) for z in zs], "expect": got})

    for n in (0, 1, 2, 3, 4, 7, 67):
        m = H(b"cert" + bytes([n]))[:32]
        items = [(pks[i], o.sign(seeds[i], m)) for i in range(n)]
        add(f"valid_n{n}", m, items, True)
        if n:
            bad = list(items)
            j = rng.randrange(n)
            sg = bytearray(bad[j][1]); sg[40] ^= 4
            bad[j] = (bad[j][0], bytes(sg))
            add(f"one_bad_s_n{n}", m, bad, False)
            bad = list(items)
            bad[j] = (bad[j][0], bytes(64))
            add(f"default_sig_n{n}", m, bad, False)
            bad = list(items)
            sg = bad[j][1]
            bad[j] = (bad[j][0], sg[:32] + (int.from_bytes(sg[32:], "little") + o.L).to_bytes(32, "little"))
            add(f"s_plus_l_n{n}", m, bad, False)
            bad = list(items)
            bad[j] = (pks[(j + 1) % 100], bad[j][1])
            add(f"wrong_key_n{n}", m, bad, False)
    # small-order A with an equation-satisfying signature: verify_strict rejects,
    # verify_batch ACCEPTS (no small-order check in dalek's batch path)
    m = H(b"cert-so")[:32]
    items = [(pks[i], o.sign(seeds[i], m)) for i in range(3)]
    ident = bytes([1]) + bytes(31)
    add("small_order_identity_A_accepted", m, items + [(ident, ident + bytes(32))], True)
    # off-curve R in the batch -> reject
    add("off_curve_R", m, items + [(pks[5], bytes([2]) + bytes(31) + bytes(32))],
        None)
    return groups


def mixed_order_pool(n=64):
    """Class 8 of SURVEY 8(d): mixed-order A = aB + T8 with a torsion-matched
    R; dalek verify_strict ACCEPTS these.  Used to seed large adversarial
    mixes (workloads.adversarial_mix) whose expected verdicts come from the
    oracle."""
    rng = random.Random(0x8888)
    T8 = torsion_gen()
    out = []
    for i in range(n):
        seed = H(b"coa-mixed" + struct.pack("<Q", i))[:32]
        m = H(b"coa-mixed-msg" + struct.pack("<Q", i))[:32]
        Ab, sg = mixed_order_signature(seed, m, T8, rng)
        assert o.verify_strict(m, Ab, sg) and sodium_verify(m, Ab, sg)
        out.append({"msg": m.hex(), "pk": Ab.hex(), "sig": sg.hex()})
    return out


def sha_vectors():
    rng = random.Random(0x5A5A)
    out = []
    for ln in (0, 1, 3, 55, 56, 63, 64, 72, 96, 111, 112, 113, 127, 128, 129, 239, 240, 255, 256, 1000, 3336, 4096 + 7):
        m = bytes(rng.getrandbits(8) for _ in range(ln))
        out.append({"msg": m.hex(), "sha512": H(m).hex()})
    return out


def main():
    files = {
        "reference_crypto.json": reference_fixtures(),
        "verify_vectors.json": verify_vectors(),
        "batch_vectors.json": batch_vectors(),
        "sha512_vectors.json": sha_vectors(),
        "mixed_order_pool.json": mixed_order_pool(),
    }
    for name, data in files.items():
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(data, f, indent=1)
        print(name, len(data))


if __name__ == "__main__":
    main()
