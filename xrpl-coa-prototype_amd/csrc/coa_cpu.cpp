// coa_cpu.cpp -- the engine's own CPU implementation of the checks its GPU
// kernels make, for a caller whose GPU calls failed.
//
// The engine's GPU entry points never fall back by themselves: with no usable
// device they return COA_ENODEVICE / COA_EHIP (coa_verify.h).  A caller that
// must keep answering -- the Rust binding under COA_ON_ENGINE_FAILURE=cpu
// (rust/crypto/src/degrade.rs), so that verdicts never depend on device
// health (SURVEY.md §5, §8(b) Errors row) -- calls the coa_cpu_* entries
// below explicitly, and counts and reports that it did.
//
// Acceptance rules are those of the pinned ed25519-dalek 1.0.1 /
// curve25519-dalek 3.x, as the GPU kernels and the test oracle state them:
//   Signature::verify       crypto/src/lib.rs:200-204 -> verify_strict:
//                           s < l (and the top 3 bits of s clear), A and R
//                           decompress (y may be >= p; negative zero kept),
//                           neither A nor R of small order, k = SHA-512(R ||
//                           A || M) mod l, accept iff [s]B - [k]A == R
//                           (projective compare, no cofactor)
//   Signature::verify_batch crypto/src/lib.rs:206-219 -> verify_batch:
//                           every s_i < l, every A_i / R_i decompresses,
//                           [-sum z_i s_i]B + sum [z_i]R_i + sum [z_i k_i]A_i
//                           is the identity (no small-order rejection, no
//                           cofactor), z_i 128-bit weights
//   Digest                  SHA-512, first 32 bytes (worker/src/processor.rs:38)
//   Certificate::verify     primary/src/messages.rs:189-215: the COA_CERT_*
//                           bits of the three crypto checks
//
// Design (host CPU, not a restatement of the oracle's): radix-2^51 field
// elements multiplied through unsigned __int128; extended twisted-Edwards
// points with the a = -1 formulas; signed radix-16 windows for every scalar,
// one shared doubling chain (Straus) for the two-term verify and for the batch
// equation; scalars reduced mod l bit-serially; the curve constants (d,
// sqrt(-1), B) derived at first use from their definitions.  Work is spread
// over std::threads in contiguous index ranges.
#include <sys/random.h>

#include <algorithm>
#include <cerrno>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "coa_verify.h"

namespace {

using u128 = unsigned __int128;
constexpr uint64_t kM51 = (uint64_t(1) << 51) - 1;

// ------------------------------------------------------------------ SHA-512
struct Sha512 {
  uint64_t st[8];
  uint8_t blk[128];
  size_t fill = 0;
  uint64_t bytes = 0;

  static uint64_t rotr(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

  Sha512() {
    static const uint64_t iv[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                                   0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                   0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
    std::memcpy(st, iv, sizeof st);
  }

  void compress(const uint8_t* p) {
    static const uint64_t rc[80] = {
        0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
        0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
        0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
        0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
        0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
        0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
        0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
        0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
        0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
        0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
        0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
        0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
        0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
        0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
        0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
        0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
        0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
        0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
        0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
        0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};
    uint64_t w[16];
    for (int i = 0; i < 16; i++) {
      uint64_t x = 0;
      for (int b = 0; b < 8; b++) x = x << 8 | p[i * 8 + b];
      w[i] = x;
    }
    uint64_t v[8];
    std::memcpy(v, st, sizeof v);
    for (int t = 0; t < 80; t++) {
      // message schedule kept in a 16-word ring
      uint64_t wt;
      if (t < 16) {
        wt = w[t];
      } else {
        const uint64_t a = w[(t + 1) & 15], b = w[(t + 14) & 15];
        wt = w[t & 15] += (rotr(a, 1) ^ rotr(a, 8) ^ (a >> 7)) + w[(t + 9) & 15] +
                          (rotr(b, 19) ^ rotr(b, 61) ^ (b >> 6));
      }
      const uint64_t e = v[4], a = v[0];
      const uint64_t t1 = v[7] + (rotr(e, 14) ^ rotr(e, 18) ^ rotr(e, 41)) + (v[6] ^ (e & (v[5] ^ v[6]))) + rc[t] + wt;
      const uint64_t t2 = (rotr(a, 28) ^ rotr(a, 34) ^ rotr(a, 39)) + ((a & v[1]) | (v[2] & (a | v[1])));
      for (int i = 7; i > 0; i--) v[i] = v[i - 1];
      v[4] += t1;
      v[0] = t1 + t2;
    }
    for (int i = 0; i < 8; i++) st[i] += v[i];
  }

  void update(const uint8_t* p, size_t n) {
    bytes += n;
    while (n) {
      if (fill == 0 && n >= 128) {
        compress(p);
        p += 128;
        n -= 128;
        continue;
      }
      const size_t k = std::min(n, 128 - fill);
      std::memcpy(blk + fill, p, k);
      fill += k;
      p += k;
      n -= k;
      if (fill == 128) {
        compress(blk);
        fill = 0;
      }
    }
  }

  void finish(uint8_t out[64]) {
    const uint64_t bits = bytes * 8;
    blk[fill++] = 0x80;
    if (fill > 112) {
      std::memset(blk + fill, 0, 128 - fill);
      compress(blk);
      fill = 0;
    }
    std::memset(blk + fill, 0, 120 - fill);  // the length's upper 64 bits are zero
    for (int b = 0; b < 8; b++) blk[120 + b] = (uint8_t)(bits >> (56 - 8 * b));
    compress(blk);
    for (int i = 0; i < 8; i++)
      for (int b = 0; b < 8; b++) out[8 * i + b] = (uint8_t)(st[i] >> (56 - 8 * b));
  }
};

void sha512(const uint8_t* p, size_t n, uint8_t out[64]) {
  Sha512 h;
  h.update(p, n);
  h.finish(out);
}

// -------------------------------------------------------- field mod 2^255-19
struct Fe {
  uint64_t v[5];
};

Fe fe_small(uint64_t x) { return Fe{{x, 0, 0, 0, 0}}; }

// limbs back under 2^51 (+ a little in limb 0)
void fe_carry(Fe& f) {
  for (int i = 0; i < 4; i++) {
    f.v[i + 1] += f.v[i] >> 51;
    f.v[i] &= kM51;
  }
  f.v[0] += 19 * (f.v[4] >> 51);
  f.v[4] &= kM51;
}

Fe fe_add(const Fe& a, const Fe& b) {
  Fe r;
  for (int i = 0; i < 5; i++) r.v[i] = a.v[i] + b.v[i];
  fe_carry(r);
  return r;
}

// a - b + 4p (limbs of b below 2^53)
Fe fe_sub(const Fe& a, const Fe& b) {
  Fe r;
  r.v[0] = a.v[0] + ((uint64_t(1) << 53) - 76) - b.v[0];
  for (int i = 1; i < 5; i++) r.v[i] = a.v[i] + ((uint64_t(1) << 53) - 4) - b.v[i];
  fe_carry(r);
  return r;
}

Fe fe_neg(const Fe& a) { return fe_sub(fe_small(0), a); }

Fe fe_mul(const Fe& a, const Fe& b) {
  const uint64_t b1 = 19 * b.v[1], b2 = 19 * b.v[2], b3 = 19 * b.v[3], b4 = 19 * b.v[4];
  const uint64_t* x = a.v;
  u128 c0 = (u128)x[0] * b.v[0] + (u128)x[1] * b4 + (u128)x[2] * b3 + (u128)x[3] * b2 + (u128)x[4] * b1;
  u128 c1 = (u128)x[0] * b.v[1] + (u128)x[1] * b.v[0] + (u128)x[2] * b4 + (u128)x[3] * b3 + (u128)x[4] * b2;
  u128 c2 = (u128)x[0] * b.v[2] + (u128)x[1] * b.v[1] + (u128)x[2] * b.v[0] + (u128)x[3] * b4 + (u128)x[4] * b3;
  u128 c3 = (u128)x[0] * b.v[3] + (u128)x[1] * b.v[2] + (u128)x[2] * b.v[1] + (u128)x[3] * b.v[0] + (u128)x[4] * b4;
  u128 c4 = (u128)x[0] * b.v[4] + (u128)x[1] * b.v[3] + (u128)x[2] * b.v[2] + (u128)x[3] * b.v[1] + (u128)x[4] * b.v[0];
  Fe r;
  c1 += (uint64_t)(c0 >> 51);
  r.v[0] = (uint64_t)c0 & kM51;
  c2 += (uint64_t)(c1 >> 51);
  r.v[1] = (uint64_t)c1 & kM51;
  c3 += (uint64_t)(c2 >> 51);
  r.v[2] = (uint64_t)c2 & kM51;
  c4 += (uint64_t)(c3 >> 51);
  r.v[3] = (uint64_t)c3 & kM51;
  r.v[4] = (uint64_t)c4 & kM51;
  r.v[0] += 19 * (uint64_t)(c4 >> 51);
  r.v[1] += r.v[0] >> 51;
  r.v[0] &= kM51;
  return r;
}

Fe fe_sq(const Fe& a) { return fe_mul(a, a); }

Fe fe_sqn(Fe a, int n) {
  while (n--) a = fe_sq(a);
  return a;
}

// 255 bits, little-endian; bit 255 ignored; values in [p, 2^255) are taken
// mod p (dalek's FieldElement::from_bytes)
Fe fe_load(const uint8_t s[32]) {
  uint64_t w[4];
  for (int i = 0; i < 4; i++) {
    w[i] = 0;
    for (int b = 7; b >= 0; b--) w[i] = w[i] << 8 | s[8 * i + b];
  }
  Fe f;
  f.v[0] = w[0] & kM51;
  f.v[1] = (w[0] >> 51 | w[1] << 13) & kM51;
  f.v[2] = (w[1] >> 38 | w[2] << 26) & kM51;
  f.v[3] = (w[2] >> 25 | w[3] << 39) & kM51;
  f.v[4] = (w[3] >> 12) & kM51;
  return f;
}

// the canonical encoding (value fully reduced below p)
void fe_store(uint8_t out[32], Fe f) {
  fe_carry(f);
  fe_carry(f);
  // f < 2^255 now; subtract p when f >= p, i.e. when f + 19 carries out of bit 255
  uint64_t q = (f.v[0] + 19) >> 51;
  for (int i = 1; i < 5; i++) q = (f.v[i] + q) >> 51;
  f.v[0] += 19 * q;
  for (int i = 0; i < 4; i++) {
    f.v[i + 1] += f.v[i] >> 51;
    f.v[i] &= kM51;
  }
  f.v[4] &= kM51;
  const uint64_t w0 = f.v[0] | f.v[1] << 51, w1 = f.v[1] >> 13 | f.v[2] << 38, w2 = f.v[2] >> 26 | f.v[3] << 25,
                 w3 = f.v[3] >> 39 | f.v[4] << 12;
  const uint64_t w[4] = {w0, w1, w2, w3};
  for (int i = 0; i < 4; i++)
    for (int b = 0; b < 8; b++) out[8 * i + b] = (uint8_t)(w[i] >> (8 * b));
}

bool fe_equal(const Fe& a, const Fe& b) {
  uint8_t x[32], y[32];
  fe_store(x, a);
  fe_store(y, b);
  return std::memcmp(x, y, 32) == 0;
}

bool fe_is_zero(const Fe& a) { return fe_equal(a, fe_small(0)); }

bool fe_is_negative(const Fe& a) {
  uint8_t x[32];
  fe_store(x, a);
  return x[0] & 1;
}

// z^(2^250 - 1) and z^11, the common prefix of the two exponent chains below
void fe_chain250(const Fe& z, Fe& z250, Fe& z11) {
  const Fe z2 = fe_sq(z);
  const Fe z9 = fe_mul(fe_sqn(z2, 2), z);
  z11 = fe_mul(z9, z2);
  const Fe e5 = fe_mul(fe_sq(z11), z9);         // 2^5 - 1
  const Fe e10 = fe_mul(fe_sqn(e5, 5), e5);     // 2^10 - 1
  const Fe e20 = fe_mul(fe_sqn(e10, 10), e10);  // 2^20 - 1
  const Fe e40 = fe_mul(fe_sqn(e20, 20), e20);  // 2^40 - 1
  const Fe e50 = fe_mul(fe_sqn(e40, 10), e10);  // 2^50 - 1
  const Fe e100 = fe_mul(fe_sqn(e50, 50), e50);
  const Fe e200 = fe_mul(fe_sqn(e100, 100), e100);
  z250 = fe_mul(fe_sqn(e200, 50), e50);
}

Fe fe_inverse(const Fe& z) {  // z^(p-2) = z^(2^255 - 21)
  Fe z250, z11;
  fe_chain250(z, z250, z11);
  return fe_mul(fe_sqn(z250, 5), z11);
}

Fe fe_pow_p58(const Fe& z) {  // z^((p-5)/8) = z^(2^252 - 3)
  Fe z250, z11;
  fe_chain250(z, z250, z11);
  return fe_mul(fe_sqn(z250, 2), z);
}

// --------------------------------------------------------- curve constants
struct Consts {
  Fe d, d2, sqrtm1;
};

struct Pt {  // extended: x = X/Z, y = Y/Z, x y = T/Z
  Fe X, Y, Z, T;
};

struct Cached {  // Y+X, Y-X, 2Z, 2dT of an addend
  Fe ypx, ymx, z2, t2d;
};

const Consts& consts();

Pt pt_identity() { return Pt{fe_small(0), fe_small(1), fe_small(1), fe_small(0)}; }

Cached pt_cache(const Pt& p) {
  const Consts& c = consts();
  return Cached{fe_add(p.Y, p.X), fe_sub(p.Y, p.X), fe_add(p.Z, p.Z), fe_mul(p.T, c.d2)};
}

// p + q (neg: p - q), a = -1 unified addition
Pt pt_add(const Pt& p, const Cached& q, bool neg) {
  const Fe a = fe_mul(fe_sub(p.Y, p.X), neg ? q.ypx : q.ymx);
  const Fe b = fe_mul(fe_add(p.Y, p.X), neg ? q.ymx : q.ypx);
  const Fe tt = fe_mul(p.T, q.t2d);
  const Fe c = neg ? fe_neg(tt) : tt;
  const Fe d = fe_mul(p.Z, q.z2);
  const Fe e = fe_sub(b, a), f = fe_sub(d, c), g = fe_add(d, c), h = fe_add(b, a);
  return Pt{fe_mul(e, f), fe_mul(g, h), fe_mul(f, g), fe_mul(e, h)};
}

Pt pt_double(const Pt& p) {
  const Fe a = fe_sq(p.X), b = fe_sq(p.Y);
  const Fe zz = fe_sq(p.Z);
  const Fe c = fe_add(zz, zz);
  const Fe e = fe_sub(fe_sub(fe_sq(fe_add(p.X, p.Y)), a), b);
  const Fe g = fe_sub(b, a);  // -a + b
  const Fe f = fe_sub(g, c);
  const Fe h = fe_neg(fe_add(a, b));  // -a - b
  return Pt{fe_mul(e, f), fe_mul(g, h), fe_mul(f, g), fe_mul(e, h)};
}

bool pt_is_identity(const Pt& p) { return fe_is_zero(p.X) && fe_equal(p.Y, p.Z); }

bool pt_same(const Pt& p, const Pt& q) {
  return fe_equal(fe_mul(p.X, q.Z), fe_mul(q.X, p.Z)) && fe_equal(fe_mul(p.Y, q.Z), fe_mul(q.Y, p.Z));
}

// [8]P == identity: the eight torsion points (P itself on the curve)
bool pt_small_order(const Pt& p) { return pt_is_identity(pt_double(pt_double(pt_double(p)))); }

// curve25519-dalek's sqrt_ratio_i: (was_square, r) with r = +sqrt(u/v) or
// +sqrt(i u/v), r non-negative
bool sqrt_ratio_i(const Fe& u, const Fe& v, Fe& r) {
  const Consts& k = consts();
  const Fe v3 = fe_mul(fe_sq(v), v);
  const Fe v7 = fe_mul(fe_sq(v3), v);
  r = fe_mul(fe_mul(u, v3), fe_pow_p58(fe_mul(u, v7)));
  const Fe check = fe_mul(v, fe_sq(r));
  const Fe mu = fe_neg(u);
  const bool correct = fe_equal(check, u), flipped = fe_equal(check, mu),
             flipped_i = fe_equal(check, fe_mul(mu, k.sqrtm1));
  if (flipped || flipped_i) r = fe_mul(r, k.sqrtm1);
  if (fe_is_negative(r)) r = fe_neg(r);
  return correct || flipped;
}

// CompressedEdwardsY::decompress: false when x^2 = (y^2 - 1) / (d y^2 + 1)
// has no root; the sign bit is applied even to x = 0
bool pt_decompress(const uint8_t s[32], Pt& p) {
  const Consts& k = consts();
  p.Y = fe_load(s);
  p.Z = fe_small(1);
  const Fe yy = fe_sq(p.Y);
  const Fe u = fe_sub(yy, p.Z);
  const Fe v = fe_add(fe_mul(yy, k.d), p.Z);
  if (!sqrt_ratio_i(u, v, p.X)) return false;
  if (s[31] >> 7) p.X = fe_neg(p.X);
  p.T = fe_mul(p.X, p.Y);
  return true;
}

Consts* g_consts = nullptr;
Pt g_base;
Cached g_base_tab[8];  // [1..8]B
std::once_flag g_once;

void init_consts() {
  static Consts c;
  // d = -121665 / 121666
  c.d = fe_mul(fe_neg(fe_small(121665)), fe_inverse(fe_small(121666)));
  c.d2 = fe_add(c.d, c.d);
  // sqrt(-1) = 2^((p-1)/4); (p-1)/4 = 2^253 - 5 = (2^250 - 1) * 8 + 3
  Fe two250, two11;
  fe_chain250(fe_small(2), two250, two11);
  c.sqrtm1 = fe_mul(fe_sqn(two250, 3), fe_mul(fe_small(2), fe_small(4)));
  g_consts = &c;
  // B: y = 4/5, x even -- the encoding 0x58 0x66 ... 0x66
  uint8_t b[32];
  std::memset(b, 0x66, 32);
  b[0] = 0x58;
  if (!pt_decompress(b, g_base)) std::abort();
  Pt m = g_base;
  for (int i = 0; i < 8; i++) {
    g_base_tab[i] = pt_cache(m);
    m = pt_add(m, g_base_tab[0], false);
  }
}

const Consts& consts() {
  if (!g_consts) std::call_once(g_once, init_consts);
  return *g_consts;
}

void ensure_consts() { (void)consts(); }

// ------------------------------------------------------------ scalars mod l
// l = 2^252 + 27742317777372353535851937790883648493, little-endian 64-bit words
constexpr uint64_t kL[4] = {0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0, 0x1000000000000000ULL};

struct Sc {
  uint64_t w[4];
};

bool sc_ge_l(const uint64_t* x) {
  for (int i = 3; i >= 0; i--)
    if (x[i] != kL[i]) return x[i] > kL[i];
  return true;
}

void sc_sub_l(uint64_t* x) {
  uint64_t borrow = 0;
  for (int i = 0; i < 4; i++) {
    const u128 t = (u128)x[i] - kL[i] - borrow;
    x[i] = (uint64_t)t;
    borrow = (uint64_t)(t >> 64) & 1;
  }
}

// an arbitrary-length little-endian integer (nw 64-bit words) mod l, one bit
// at a time from the top: r = 2r + bit, minus l when r >= l (r < 2l < 2^254)
Sc sc_mod(const uint64_t* x, int nw) {
  Sc r{{0, 0, 0, 0}};
  for (int i = nw * 64 - 1; i >= 0; i--) {
    const uint64_t bit = x[i / 64] >> (i % 64) & 1;
    r.w[3] = r.w[3] << 1 | r.w[2] >> 63;
    r.w[2] = r.w[2] << 1 | r.w[1] >> 63;
    r.w[1] = r.w[1] << 1 | r.w[0] >> 63;
    r.w[0] = r.w[0] << 1 | bit;
    if (sc_ge_l(r.w)) sc_sub_l(r.w);
  }
  return r;
}

void load_words(uint64_t* w, const uint8_t* s, int nw) {
  for (int i = 0; i < nw; i++) {
    w[i] = 0;
    for (int b = 7; b >= 0; b--) w[i] = w[i] << 8 | s[8 * i + b];
  }
}

Sc sc_from_hash(const uint8_t h[64]) {
  uint64_t w[8];
  load_words(w, h, 8);
  return sc_mod(w, 8);
}

Sc sc_mul(const Sc& a, const Sc& b) {
  uint64_t p[8] = {0};
  for (int i = 0; i < 4; i++) {
    u128 carry = 0;
    for (int j = 0; j < 4; j++) {
      carry += (u128)a.w[i] * b.w[j] + p[i + j];
      p[i + j] = (uint64_t)carry;
      carry >>= 64;
    }
    p[i + 4] = (uint64_t)carry;
  }
  return sc_mod(p, 8);
}

Sc sc_add(const Sc& a, const Sc& b) {  // a, b < l
  Sc r;
  u128 c = 0;
  for (int i = 0; i < 4; i++) {
    c += (u128)a.w[i] + b.w[i];
    r.w[i] = (uint64_t)c;
    c >>= 64;
  }
  if (sc_ge_l(r.w)) sc_sub_l(r.w);
  return r;
}

Sc sc_negate(const Sc& a) {  // l - a (0 stays 0)
  if ((a.w[0] | a.w[1] | a.w[2] | a.w[3]) == 0) return a;
  Sc r;
  uint64_t borrow = 0;
  for (int i = 0; i < 4; i++) {
    const u128 t = (u128)kL[i] - a.w[i] - borrow;
    r.w[i] = (uint64_t)t;
    borrow = (uint64_t)(t >> 64) & 1;
  }
  return r;
}

// signed radix-16 digits in [-8, 8]: 64 digits for a scalar below 2^255
void sc_digits16(const Sc& s, int8_t d[64]) {
  for (int i = 0; i < 64; i++) d[i] = (int8_t)(s.w[i / 16] >> (4 * (i % 16)) & 15);
  int carry = 0;
  for (int i = 0; i < 63; i++) {
    int x = d[i] + carry;
    carry = (x + 8) >> 4;
    d[i] = (int8_t)(x - (carry << 4));
  }
  d[63] = (int8_t)(d[63] + carry);
}

// [1..8]P
void pt_table(const Pt& p, Cached tab[8]) {
  tab[0] = pt_cache(p);
  Pt m = p;
  for (int i = 1; i < 8; i++) {
    m = pt_add(m, tab[0], false);
    tab[i] = pt_cache(m);
  }
}

void add_digit(Pt& q, const Cached* tab, int d) {
  if (d > 0) q = pt_add(q, tab[d - 1], false);
  if (d < 0) q = pt_add(q, tab[-d - 1], true);
}

// sum_i [sc_i] P_i over tables of [1..8]P_i: Straus, one shared chain of
// doublings, 4 bits per step
Pt straus(const std::vector<const Cached*>& tabs, const std::vector<Sc>& scs) {
  const size_t n = tabs.size();
  std::vector<int8_t> dig(n * 64);
  for (size_t j = 0; j < n; j++) sc_digits16(scs[j], &dig[j * 64]);
  Pt q = pt_identity();
  for (int i = 63; i >= 0; i--) {
    if (i != 63)
      for (int k = 0; k < 4; k++) q = pt_double(q);
    for (size_t j = 0; j < n; j++) add_digit(q, tabs[j], dig[j * 64 + i]);
  }
  return q;
}

bool scalar_canonical(const uint8_t s[32], Sc& out) {
  if (s[31] & 0xe0) return false;  // ed25519::Signature::from_bytes (dalek 1.0.1 check_scalar)
  load_words(out.w, s, 4);
  return !sc_ge_l(out.w);
}

Sc challenge(const uint8_t* R, const uint8_t* A, const uint8_t* msg, size_t msg_len) {
  Sha512 h;
  h.update(R, 32);
  h.update(A, 32);
  h.update(msg, msg_len);
  uint8_t d[64];
  h.finish(d);
  return sc_from_hash(d);
}

// ed25519-dalek 1.0.1 PublicKey::verify_strict: 0 Ok / 1 Err
int verify_strict_one(const uint8_t* msg, size_t msg_len, const uint8_t* pk, const uint8_t* sig) {
  Sc s;
  if (!scalar_canonical(sig + 32, s)) return 1;
  Pt A, R;
  if (!pt_decompress(pk, A) || !pt_decompress(sig, R)) return 1;
  if (pt_small_order(A) || pt_small_order(R)) return 1;
  const Sc k = challenge(sig, pk, msg, msg_len);
  Cached atab[8];
  pt_table(A, atab);
  // [s]B - [k]A: the A digits negated
  int8_t ds[64], dk[64];
  sc_digits16(s, ds);
  sc_digits16(k, dk);
  Pt q = pt_identity();
  for (int i = 63; i >= 0; i--) {
    if (i != 63)
      for (int j = 0; j < 4; j++) q = pt_double(q);
    add_digit(q, g_base_tab, ds[i]);
    add_digit(q, atab, -dk[i]);
  }
  return pt_same(q, R) ? 0 : 1;
}

// ed25519-dalek 1.0.1 verify_batch over one message: 0 Ok / 1 Err; zs: 16
// little-endian bytes per signature
int verify_batch_one(const uint8_t* msg, size_t msg_len, const uint8_t* pks, const uint8_t* sigs, size_t n,
                     const uint8_t* zs) {
  std::vector<Cached> tabs((2 * n) * 8);
  std::vector<const Cached*> tp;
  std::vector<Sc> sc;
  tp.reserve(2 * n + 1);
  sc.reserve(2 * n + 1);
  Sc bsum{{0, 0, 0, 0}};
  tp.push_back(g_base_tab);
  sc.push_back(bsum);  // the B coefficient, set below
  for (size_t i = 0; i < n; i++) {
    const uint8_t* sig = sigs + 64 * i;
    const uint8_t* pk = pks + 32 * i;
    Sc s;
    if (!scalar_canonical(sig + 32, s)) return 1;
    Pt A, R;
    if (!pt_decompress(pk, A) || !pt_decompress(sig, R)) return 1;
    Sc z{{0, 0, 0, 0}};
    load_words(z.w, zs + 16 * i, 2);
    bsum = sc_add(bsum, sc_mul(z, s));
    pt_table(R, &tabs[(2 * i) * 8]);
    pt_table(A, &tabs[(2 * i + 1) * 8]);
    tp.push_back(&tabs[(2 * i) * 8]);
    sc.push_back(z);
    tp.push_back(&tabs[(2 * i + 1) * 8]);
    sc.push_back(sc_mul(z, challenge(sig, pk, msg, msg_len)));
  }
  sc[0] = sc_negate(bsum);
  return pt_is_identity(straus(tp, sc)) ? 0 : 1;
}

bool os_random(uint8_t* p, size_t n) {
  while (n) {
    const ssize_t k = getrandom(p, n, 0);
    if (k < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += k;
    n -= (size_t)k;
  }
  return true;
}

// weights from rng_seed (0 = OS entropy): SHA-512 in counter mode over the
// seed when one is given (reproducible)
bool make_weights(uint8_t* zs, size_t n, uint64_t rng_seed) {
  if (rng_seed == 0) return os_random(zs, 16 * n);
  uint8_t in[16], out[64];
  for (int b = 0; b < 8; b++) in[b] = (uint8_t)(rng_seed >> (8 * b));
  for (size_t i = 0; i < n; i += 4) {
    const uint64_t ctr = i;
    for (int b = 0; b < 8; b++) in[8 + b] = (uint8_t)(ctr >> (8 * b));
    sha512(in, 16, out);
    std::memcpy(zs + 16 * i, out, 16 * std::min<size_t>(4, n - i));
  }
  return true;
}

int threads_for(size_t items, int nthreads) {
  if (nthreads <= 0) {
    const unsigned hc = std::thread::hardware_concurrency();
    nthreads = (int)std::min<unsigned>(hc ? hc : 1, 16);
  }
  return (int)std::max<size_t>(1, std::min<size_t>((size_t)nthreads, items));
}

// fn(lo, hi) over contiguous ranges of [0, n) on nthreads threads
template <class F>
void parallel_ranges(size_t n, int nthreads, F fn) {
  const int t = threads_for(n, nthreads);
  if (t == 1) {
    fn((size_t)0, n);
    return;
  }
  std::vector<std::thread> th;
  th.reserve((size_t)t);
  for (int i = 0; i < t; i++) th.emplace_back(fn, n * (size_t)i / (size_t)t, n * (size_t)(i + 1) / (size_t)t);
  for (auto& x : th) x.join();
}

struct CertView {
  const uint8_t *hdata, *ids, *origins, *hsigs, *vpks, *vsigs;
  const uint64_t *hoff, *rounds, *voff;
};

// COA_CERT_* bits of one certificate (the engine's status semantics)
uint8_t certificate_bits(const CertView& c, size_t i, const uint8_t* zs_all) {
  uint8_t bits = 0, h[64], m[72];
  sha512(c.hdata + c.hoff[i], (size_t)(c.hoff[i + 1] - c.hoff[i]), h);
  if (std::memcmp(h, c.ids + 32 * i, 32) != 0) bits |= COA_CERT_BAD_HEADER_ID;
  if (verify_strict_one(c.ids + 32 * i, 32, c.origins + 32 * i, c.hsigs + 64 * i)) bits |= COA_CERT_BAD_HEADER_SIG;
  // Certificate::digest = SHA-512(id || round LE || origin)[..32] (messages.rs:226-234)
  std::memcpy(m, c.ids + 32 * i, 32);
  for (int b = 0; b < 8; b++) m[32 + b] = (uint8_t)(c.rounds[i] >> (8 * b));
  std::memcpy(m + 40, c.origins + 32 * i, 32);
  sha512(m, 72, h);
  const uint64_t v0 = c.voff[i], nv = c.voff[i + 1] - v0;
  if (verify_batch_one(h, 32, c.vpks + 32 * v0, c.vsigs + 64 * v0, (size_t)nv, zs_all + 16 * v0))
    bits |= COA_CERT_BAD_VOTES;
  return bits;
}

}  // namespace

extern "C" {

int coa_cpu_ed25519_verify_strict(const uint8_t* msg, size_t msg_len, const uint8_t pk[32], const uint8_t sig[64]) {
  if ((!msg && msg_len) || !pk || !sig) return COA_EINVAL;
  ensure_consts();
  return verify_strict_one(msg, msg_len, pk, sig);
}

int coa_cpu_ed25519_verify_strict_many(const uint8_t* msgs, size_t msg_len, const uint8_t* pks, const uint8_t* sigs,
                                       size_t n, uint8_t* verdicts_out, int nthreads) {
  if (n == 0) return COA_OK;
  if ((!msgs && msg_len) || !pks || !sigs || !verdicts_out) return COA_EINVAL;
  ensure_consts();
  parallel_ranges(n, nthreads, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; i++)
      verdicts_out[i] = (uint8_t)verify_strict_one(msgs + i * msg_len, msg_len, pks + 32 * i, sigs + 64 * i);
  });
  return COA_OK;
}

int coa_cpu_ed25519_verify_batch_groups_z(const uint8_t* msgs, const uint8_t* pks, const uint8_t* sigs,
                                          const uint64_t* group_offsets, size_t n_groups, const uint8_t* zs,
                                          uint8_t* group_verdicts_out, int nthreads) {
  if (n_groups == 0) return COA_OK;
  if (!msgs || !group_offsets || !group_verdicts_out || group_offsets[0] != 0) return COA_EINVAL;
  const uint64_t total = group_offsets[n_groups];
  for (size_t g = 0; g < n_groups; g++)
    if (group_offsets[g + 1] < group_offsets[g]) return COA_EINVAL;
  if (total && (!pks || !sigs || !zs)) return COA_EINVAL;
  ensure_consts();
  parallel_ranges(n_groups, nthreads, [&](size_t lo, size_t hi) {
    for (size_t g = lo; g < hi; g++) {
      const uint64_t a = group_offsets[g], b = group_offsets[g + 1];
      group_verdicts_out[g] =
          (uint8_t)verify_batch_one(msgs + 32 * g, 32, pks + 32 * a, sigs + 64 * a, (size_t)(b - a), zs + 16 * a);
    }
  });
  return COA_OK;
}

int coa_cpu_ed25519_verify_batch(const uint8_t msg[32], const uint8_t* pks, const uint8_t* sigs, size_t n,
                                 uint64_t rng_seed) {
  if (!msg || (n && (!pks || !sigs))) return COA_EINVAL;
  std::vector<uint8_t> zs(16 * n + 16);
  if (!make_weights(zs.data(), n, rng_seed)) return COA_EINVAL;
  const uint64_t off[2] = {0, n};
  uint8_t v = 1;
  const int rc = coa_cpu_ed25519_verify_batch_groups_z(msg, pks, sigs, off, 1, zs.data(), &v, 1);
  return rc != COA_OK ? rc : v;
}

int coa_cpu_sha512_many(const uint8_t* data, const uint64_t* offsets, size_t n, uint8_t* out64, int nthreads) {
  if (n == 0) return COA_OK;
  if (!offsets || !out64 || (!data && offsets[n] > offsets[0])) return COA_EINVAL;
  for (size_t i = 0; i < n; i++)
    if (offsets[i + 1] < offsets[i]) return COA_EINVAL;
  parallel_ranges(n, nthreads, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; i++) sha512(data + offsets[i], (size_t)(offsets[i + 1] - offsets[i]), out64 + 64 * i);
  });
  return COA_OK;
}

int coa_cpu_certificate_verify_many_z(const uint8_t* header_data, const uint64_t* header_offsets, const uint8_t* ids,
                                      const uint8_t* origins, const uint8_t* header_sigs, const uint64_t* rounds,
                                      const uint8_t* vote_pks, const uint8_t* vote_sigs, const uint64_t* vote_offsets,
                                      size_t n, const uint8_t* zs, uint8_t* status_out, int nthreads) {
  if (n == 0) return COA_OK;
  if (!header_offsets || !ids || !origins || !header_sigs || !rounds || !vote_offsets || !status_out ||
      vote_offsets[0] != 0)
    return COA_EINVAL;
  for (size_t i = 0; i < n; i++)
    if (header_offsets[i + 1] < header_offsets[i] || vote_offsets[i + 1] < vote_offsets[i]) return COA_EINVAL;
  if (header_offsets[n] > header_offsets[0] && !header_data) return COA_EINVAL;
  if (vote_offsets[n] && (!vote_pks || !vote_sigs || !zs)) return COA_EINVAL;
  ensure_consts();
  const CertView c{header_data, ids, origins, header_sigs, vote_pks, vote_sigs, header_offsets, rounds, vote_offsets};
  parallel_ranges(n, nthreads, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; i++) status_out[i] = certificate_bits(c, i, zs);
  });
  return COA_OK;
}

int coa_cpu_certificate_verify_many(const uint8_t* header_data, const uint64_t* header_offsets, const uint8_t* ids,
                                    const uint8_t* origins, const uint8_t* header_sigs, const uint64_t* rounds,
                                    const uint8_t* vote_pks, const uint8_t* vote_sigs, const uint64_t* vote_offsets,
                                    size_t n, uint64_t rng_seed, uint8_t* status_out, int nthreads) {
  if (n == 0) return COA_OK;
  if (!vote_offsets) return COA_EINVAL;
  std::vector<uint8_t> zs(16 * vote_offsets[n] + 16);
  if (!make_weights(zs.data(), (size_t)vote_offsets[n], rng_seed)) return COA_EINVAL;
  return coa_cpu_certificate_verify_many_z(header_data, header_offsets, ids, origins, header_sigs, rounds, vote_pks,
                                           vote_sigs, vote_offsets, n, zs.data(), status_out, nthreads);
}

}  // extern "C"
