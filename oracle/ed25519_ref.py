"""CPU ORACLE -- test infrastructure only.

Pure-Python big-integer restatement of the arithmetic behind the reference's
`crypto` crate hot path (`crypto/src/lib.rs:200-219`):

* `Signature::verify`  -> ed25519-dalek 1.0.1 `PublicKey::verify_strict`
* `Signature::verify_batch` -> ed25519-dalek 1.0.1 `verify_batch` (feature "batch")
* `Digest`             -> sha2 0.9 `Sha512::digest(..)[..32]`

The arithmetic itself lives in third-party crates that are NOT vendored in
/root/reference (no Cargo.lock, `.gitignore:20`): ed25519-dalek 1.0.1,
curve25519-dalek 3.x (u64 backend), ed25519 1.x, sha2 0.9.  Their published
algorithms are restated here; each function names the dalek routine whose
acceptance behaviour it reproduces.  Parity anchors: the reference's own call
sites (`crypto/src/lib.rs:201-203,215-218`) and tests
(`crypto/src/tests/crypto_tests.rs:49-115`), RFC 8032 known answers and
libsodium 1.0.18 cross-checks (see tests/golden/make_golden.py).

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s cpu_baseline leg may
import this module, and only as the checker.  Sizes: small cases only (each
verify is a few milliseconds of pure Python).
"""
import hashlib

P = 2 ** 255 - 19
L = 2 ** 252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
D2 = (2 * D) % P
SQRT_M1 = pow(2, (P - 1) // 4, P)

# Base point (RFC 8032 5.1): y = 4/5, x positive (even).
_BY = (4 * pow(5, P - 2, P)) % P


def _recover_x(y, sign):
    u = (y * y - 1) % P
    v = (D * y * y + 1) % P
    ok, x = sqrt_ratio_i(u, v)
    assert ok
    if sign:
        x = (-x) % P
    return x


def is_negative(x):
    """curve25519-dalek FieldElement::is_negative: low bit of canonical bytes."""
    return (x % P) & 1


def sqrt_ratio_i(u, v):
    """curve25519-dalek 3.x field.rs `FieldElement::sqrt_ratio_i`.

    Returns (was_nonzero_square, r) with r the NON-NEGATIVE root of u/v, or of
    i*u/v when u/v is a non-square.  u == 0 yields (True, 0).
    """
    u %= P
    v %= P
    v3 = v * v % P * v % P
    v7 = v3 * v3 % P * v % P
    r = (u * v3 % P) * pow(u * v7 % P, (P - 5) // 8, P) % P
    check = v * r % P * r % P
    correct_sign = check == u
    flipped_sign = check == (-u) % P
    flipped_sign_i = check == (-u * SQRT_M1) % P
    if flipped_sign or flipped_sign_i:
        r = r * SQRT_M1 % P
    if is_negative(r):
        r = (-r) % P
    return (correct_sign or flipped_sign), r


# ---------------------------------------------------------------------------
# Points: extended homogeneous (X:Y:Z:T), x=X/Z, y=Y/Z, xy=T/Z.
# The a=-1 twisted-Edwards addition law below is complete for d non-square,
# so it is exact for every point, torsion included.
# ---------------------------------------------------------------------------
IDENT = (0, 1, 1, 0)


def padd(p, q):
    X1, Y1, Z1, T1 = p
    X2, Y2, Z2, T2 = q
    a = (Y1 - X1) * (Y2 - X2) % P
    b = (Y1 + X1) * (Y2 + X2) % P
    c = T1 * D2 % P * T2 % P
    d = Z1 * 2 * Z2 % P
    e, f, g, h = b - a, d - c, d + c, b + a
    return (e * f % P, g * h % P, f * g % P, e * h % P)


def pdbl(p):
    return padd(p, p)


def pneg(p):
    X, Y, Z, T = p
    return ((-X) % P, Y, Z, (-T) % P)


def pmul(k, p):
    """[k]p for k >= 0 (plain double-and-add; any exact algorithm gives the
    same group element as dalek's w-NAF/Straus/Pippenger)."""
    r = IDENT
    for bit in bin(k)[2:] if k > 0 else "":
        r = pdbl(r)
        if bit == "1":
            r = padd(r, p)
    return r


def peq(p, q):
    """curve25519-dalek EdwardsPoint::ct_eq: projective X1Z2==X2Z1, Y1Z2==Y2Z1."""
    X1, Y1, Z1, _ = p
    X2, Y2, Z2, _ = q
    return (X1 * Z2 - X2 * Z1) % P == 0 and (Y1 * Z2 - Y2 * Z1) % P == 0


def is_identity(p):
    return peq(p, IDENT)


def is_small_order(p):
    """curve25519-dalek EdwardsPoint::is_small_order: [8]p == identity."""
    return is_identity(pdbl(pdbl(pdbl(p))))


def compress(p):
    X, Y, Z, _ = p
    zi = pow(Z, P - 2, P)
    x, y = X * zi % P, Y * zi % P
    return (y | (is_negative(x) << 255)).to_bytes(32, "little")


B = (_recover_x(_BY, 0), _BY, 1, _recover_x(_BY, 0) * _BY % P)


def decompress(b):
    """curve25519-dalek 3.x CompressedEdwardsY::decompress.

    * y is read as 255 bits (bit 255 masked) and is NOT required to be < p:
      FieldElement51::from_bytes keeps y in [p, 2^255) unreduced, so such an
      encoding means y - p.
    * sqrt_ratio_i(y^2-1, d*y^2+1) must report a square (zero counts).
    * x is negated by the sign bit even when x == 0 ("negative zero").
    Returns an extended point or None.
    """
    assert len(b) == 32
    y = (int.from_bytes(b, "little") & ((1 << 255) - 1)) % P
    u = (y * y - 1) % P
    v = (D * y * y + 1) % P
    ok, x = sqrt_ratio_i(u, v)
    if not ok:
        return None
    if b[31] >> 7:
        x = (-x) % P
    return (x, y, 1, x * y % P)


def sha512(data):
    return hashlib.sha512(bytes(data)).digest()


def digest32(data):
    """crypto::Digest as computed at primary/src/messages.rs:72-82 and
    worker/src/processor.rs:38: Sha512(bytes)[..32]."""
    return sha512(data)[:32]


def scalar_from_hash(h):
    """curve25519-dalek Scalar::from_hash: 64-byte LE value mod l."""
    return int.from_bytes(h, "little") % L


def scalar_is_canonical(sb):
    """ed25519-dalek 1.0.1 `check_scalar` (default features) ==
    Scalar::from_canonical_bytes: s < l.  The ed25519 1.x `from_bytes`
    top-3-bit test is implied by it."""
    return int.from_bytes(sb, "little") < L


# ---------------------------------------------------------------------------
# crypto::Signature::verify (crypto/src/lib.rs:200-204)
# ---------------------------------------------------------------------------
def verify_strict(msg, pk, sig):
    """Returns True iff `Signature::verify(digest=msg, public_key=pk)` is Ok.

    Order of checks follows crypto/src/lib.rs:201-203 then dalek 1.0.1
    `verify_strict`; every failure is the same opaque error, so only the
    boolean matters.
    """
    if len(sig) != 64 or len(pk) != 32:
        return False
    # ed25519::Signature::from_bytes + InternalSignature::try_from (check_scalar)
    if sig[63] & 0xE0:
        return False
    if not scalar_is_canonical(sig[32:]):
        return False
    A = decompress(pk)  # dalek::PublicKey::from_bytes
    if A is None:
        return False
    R = decompress(sig[:32])
    if R is None:
        return False
    if is_small_order(R) or is_small_order(A):
        return False
    k = scalar_from_hash(sha512(bytes(sig[:32]) + bytes(pk) + bytes(msg)))
    s = int.from_bytes(sig[32:], "little")
    Rp = padd(pmul(k, pneg(A)), pmul(s, B))  # vartime_double_scalar_mul_basepoint(k, -A, s)
    return peq(Rp, R)


def verify_equation_cofactorless(msg, pk, sig):
    """[s]B - [k]A == R without the small-order rejection (the per-signature
    condition that verify_batch's random linear combination tests)."""
    if not scalar_is_canonical(sig[32:]) or sig[63] & 0xE0:
        return False
    A = decompress(pk)
    R = decompress(sig[:32])
    if A is None or R is None:
        return False
    k = scalar_from_hash(sha512(bytes(sig[:32]) + bytes(pk) + bytes(msg)))
    s = int.from_bytes(sig[32:], "little")
    return peq(padd(pmul(k, pneg(A)), pmul(s, B)), R)


# ---------------------------------------------------------------------------
# crypto::Signature::verify_batch (crypto/src/lib.rs:206-219)
# ---------------------------------------------------------------------------
def verify_batch(msg, pks, sigs, zs):
    """dalek 1.0.1 `verify_batch` with the 128-bit random weights `zs` given
    explicitly (dalek draws them from a merlin transcript + thread_rng).

    Ok iff every s_i < l, every A_i and R_i decompresses, and
      [-(sum z_i s_i mod l)]B + sum [z_i]R_i + sum [z_i*H(R_i||A_i||M) mod l]A_i
    is the identity.  No small-order rejection, no cofactor.
    An empty batch is Ok (the sum is [0]B).
    """
    assert len(pks) == len(sigs) == len(zs)
    pts = []
    for pk, sig in zip(pks, sigs):  # crypto/src/lib.rs:213-217
        if len(sig) != 64 or sig[63] & 0xE0:
            return False
        A = decompress(pk)
        if A is None:
            return False
        pts.append(A)
    hrams, ss = [], []
    for pk, sig in zip(pks, sigs):
        if not scalar_is_canonical(sig[32:]):
            return False
        ss.append(int.from_bytes(sig[32:], "little"))
        hrams.append(scalar_from_hash(sha512(bytes(sig[:32]) + bytes(pk) + bytes(msg))))
    Rs = []
    for sig in sigs:
        R = decompress(sig[:32])
        if R is None:
            return False
        Rs.append(R)
    bcoef = (-sum(z * s for z, s in zip(zs, ss))) % L
    acc = pmul(bcoef, B)
    for z, h, R, A in zip(zs, hrams, Rs, pts):
        acc = padd(acc, pmul(z, R))
        acc = padd(acc, pmul(z * h % L, A))
    return is_identity(acc)


# ---------------------------------------------------------------------------
# RFC 8032 signing (== dalek 1.0.1 ExpandedSecretKey::sign; fixtures only)
# ---------------------------------------------------------------------------
def expand_seed(seed):
    h = sha512(seed)
    a = bytearray(h[:32])
    a[0] &= 248
    a[31] &= 127
    a[31] |= 64
    return int.from_bytes(a, "little"), h[32:]


def public_key(seed):
    a, _ = expand_seed(seed)
    return compress(pmul(a, B))


def sign(seed, msg):
    a, prefix = expand_seed(seed)
    A = compress(pmul(a, B))
    r = scalar_from_hash(sha512(prefix + bytes(msg)))
    R = compress(pmul(r, B))
    k = scalar_from_hash(sha512(R + A + bytes(msg)))
    s = (r + k * a) % L
    return R + s.to_bytes(32, "little")


# Small-order points: the 8 torsion points E[8].
def torsion_points():
    """All 8 points of order dividing 8, as extended points."""
    # order-8 generator: a point T8 with [8]T8 = O and [4]T8 != O.
    pts = []
    for y in range(0, 64):
        pass
    # Construct from y of order-8 point: solve via sqrt.
    # Points of order 4: (+-sqrt(-1), 0); order 2: (0, -1); identity (0, 1).
    # Order 8 points have x^2 = ... ; find them by halving an order-4 point:
    # take generic approach: [l]P for random P lands in E[8].
    seen = {}
    y = 2
    while len(seen) < 8:
        b = y.to_bytes(32, "little")
        Pt = decompress(b)
        if Pt is not None:
            Tt = pmul(L, Pt)
            # generate the subgroup spanned by Tt
            cur = IDENT
            for _ in range(8):
                seen[compress(cur)] = cur
                cur = padd(cur, Tt)
        y += 1
    return list(seen.values())


def small_order_encodings():
    """Every 32-byte encoding that decompresses to a small-order point:
    canonical encodings with both sign bits, plus non-canonical y >= p
    encodings (y + p < 2^255) -- dalek accepts all of them at decompression."""
    out = []
    for T in torsion_points():
        c = bytearray(compress(T))
        y = int.from_bytes(c, "little") & ((1 << 255) - 1)
        for yy in (y, y + P):
            if yy >= 1 << 255:
                continue
            for sgn in (0, 1):
                enc = (yy | (sgn << 255)).to_bytes(32, "little")
                if decompress(enc) is not None and enc not in out:
                    out.append(enc)
    return out
