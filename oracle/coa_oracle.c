/*
 * CPU ORACLE -- test infrastructure and CPU baseline only.
 *
 * Plain-C restatement of the algorithms the reference's crypto hot path runs
 * inside its (un-vendored) third-party crates:
 *   ed25519-dalek 1.0.1  PublicKey::verify_strict, verify_batch (feature batch)
 *   curve25519-dalek 3.x u64 backend: radix-2^51 FieldElement51,
 *                        CompressedEdwardsY::decompress, is_small_order,
 *                        vartime_double_scalar_mul_basepoint (w-NAF 5 for A,
 *                        w-NAF 8 over a precomputed table of odd multiples
 *                        of B), Straus vartime multiscalar multiplication
 *   sha2 0.9             Sha512
 * as called from crypto/src/lib.rs:200-219.  Semantics (acceptance rules) are
 * identical to oracle/ed25519_ref.py; the golden fixtures in tests/golden/
 * pin both.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load the shared library built from this file.
 *
 * Build: oracle/Makefile -> oracle/_build/libcoa_oracle.so and
 * libcoa_oracle_count.so (-DCOA_COUNT: counts field multiplications and
 * squarings to freeze the algorithmic work per verification).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

#ifdef COA_COUNT
static __thread uint64_t g_nmul, g_nsq;
#define CNT_MUL (g_nmul++)
#define CNT_SQ (g_nsq++)
#else
#define CNT_MUL ((void)0)
#define CNT_SQ ((void)0)
#endif

/* ================================================================ SHA-512 */
static const uint64_t K[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL, 0x3956c25bf348b538ULL,
    0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL, 0xd807aa98a3030242ULL, 0x12835b0145706fbeULL,
    0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL, 0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL,
    0xc19bf174cf692694ULL, 0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL, 0x983e5152ee66dfabULL,
    0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL, 0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL,
    0x06ca6351e003826fULL, 0x142929670a0e6e70ULL, 0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL,
    0x53380d139d95b3dfULL, 0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL, 0xd192e819d6ef5218ULL,
    0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL, 0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL,
    0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL, 0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL,
    0x682e6ff3d6b2b8a3ULL, 0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL, 0xca273eceea26619cULL,
    0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL, 0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL,
    0x113f9804bef90daeULL, 0x1b710b35131c471bULL, 0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL,
    0x431d67c49c100d4cULL, 0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

typedef struct {
  uint64_t h[8];
  uint8_t buf[128];
  size_t nbuf;
  uint64_t total;
} sha512_ctx;

#define ROR(x, n) (((x) >> (n)) | ((x) << (64 - (n))))

static void sha512_block(uint64_t* h, const uint8_t* p) {
  uint64_t w[80];
  for (int t = 0; t < 16; t++) {
    uint64_t x = 0;
    for (int b = 0; b < 8; b++) x = (x << 8) | p[8 * t + b];
    w[t] = x;
  }
  for (int t = 16; t < 80; t++) {
    uint64_t s0 = ROR(w[t - 15], 1) ^ ROR(w[t - 15], 8) ^ (w[t - 15] >> 7);
    uint64_t s1 = ROR(w[t - 2], 19) ^ ROR(w[t - 2], 61) ^ (w[t - 2] >> 6);
    w[t] = w[t - 16] + s0 + w[t - 7] + s1;
  }
  uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int t = 0; t < 80; t++) {
    uint64_t t1 = hh + (ROR(e, 14) ^ ROR(e, 18) ^ ROR(e, 41)) + ((e & f) ^ (~e & g)) + K[t] + w[t];
    uint64_t t2 = (ROR(a, 28) ^ ROR(a, 34) ^ ROR(a, 39)) + ((a & b) ^ (a & c) ^ (b & c));
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

static void sha512_init(sha512_ctx* c) {
  static const uint64_t iv[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                                 0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
  memcpy(c->h, iv, sizeof iv);
  c->nbuf = 0;
  c->total = 0;
}

static void sha512_update(sha512_ctx* c, const uint8_t* p, size_t n) {
  c->total += n;
  if (c->nbuf) {
    size_t take = 128 - c->nbuf;
    if (take > n) take = n;
    memcpy(c->buf + c->nbuf, p, take);
    c->nbuf += take;
    p += take;
    n -= take;
    if (c->nbuf == 128) {
      sha512_block(c->h, c->buf);
      c->nbuf = 0;
    }
  }
  while (n >= 128) {
    sha512_block(c->h, p);
    p += 128;
    n -= 128;
  }
  if (n) {
    memcpy(c->buf, p, n);
    c->nbuf = n;
  }
}

static void sha512_final(sha512_ctx* c, uint8_t out[64]) {
  uint64_t bits = c->total * 8;
  uint8_t pad = 0x80;
  sha512_update(c, &pad, 1);
  uint8_t z = 0;
  while (c->nbuf != 112) sha512_update(c, &z, 1);
  uint8_t len[16] = {0};
  for (int i = 0; i < 8; i++) len[15 - i] = (uint8_t)(bits >> (8 * i));
  sha512_update(c, len, 16);
  for (int i = 0; i < 8; i++)
    for (int b = 0; b < 8; b++) out[8 * i + b] = (uint8_t)(c->h[i] >> (56 - 8 * b));
}

void coa_oracle_sha512(const uint8_t* p, size_t n, uint8_t out[64]) {
  sha512_ctx c;
  sha512_init(&c);
  sha512_update(&c, p, n);
  sha512_final(&c, out);
}

void coa_oracle_sha512_many(const uint8_t* data, const uint64_t* off, size_t n, uint8_t* out64) {
  for (size_t i = 0; i < n; i++) coa_oracle_sha512(data + off[i], off[i + 1] - off[i], out64 + 64 * i);
}

/* ============================================================= field 2^51 */
typedef struct {
  uint64_t v[5];
} fe;
#define M51 ((1ULL << 51) - 1)

static void fe_carry(fe* r) {
  uint64_t c;
  c = r->v[0] >> 51; r->v[0] &= M51; r->v[1] += c;
  c = r->v[1] >> 51; r->v[1] &= M51; r->v[2] += c;
  c = r->v[2] >> 51; r->v[2] &= M51; r->v[3] += c;
  c = r->v[3] >> 51; r->v[3] &= M51; r->v[4] += c;
  c = r->v[4] >> 51; r->v[4] &= M51; r->v[0] += c * 19;
}
static void fe_0(fe* r) { memset(r, 0, sizeof *r); }
static void fe_1(fe* r) { fe_0(r); r->v[0] = 1; }
static void fe_add(fe* r, const fe* a, const fe* b) {
  for (int i = 0; i < 5; i++) r->v[i] = a->v[i] + b->v[i];
  fe_carry(r);
}
/* a - b = a + 4p - b (limbs of b < 2^53) */
static void fe_sub(fe* r, const fe* a, const fe* b) {
  r->v[0] = a->v[0] + 0x1fffffffffffb4ULL - b->v[0];
  for (int i = 1; i < 5; i++) r->v[i] = a->v[i] + 0x1ffffffffffffcULL - b->v[i];
  fe_carry(r);
}
static void fe_neg(fe* r, const fe* a) {
  fe z;
  fe_0(&z);
  fe_sub(r, &z, a);
}
static void fe_mul(fe* r, const fe* a, const fe* b) {
  CNT_MUL;
  const uint64_t a0 = a->v[0], a1 = a->v[1], a2 = a->v[2], a3 = a->v[3], a4 = a->v[4];
  const uint64_t b0 = b->v[0], b1 = b->v[1], b2 = b->v[2], b3 = b->v[3], b4 = b->v[4];
  const uint64_t b1_19 = b1 * 19, b2_19 = b2 * 19, b3_19 = b3 * 19, b4_19 = b4 * 19;
  u128 c0 = (u128)a0 * b0 + (u128)a1 * b4_19 + (u128)a2 * b3_19 + (u128)a3 * b2_19 + (u128)a4 * b1_19;
  u128 c1 = (u128)a0 * b1 + (u128)a1 * b0 + (u128)a2 * b4_19 + (u128)a3 * b3_19 + (u128)a4 * b2_19;
  u128 c2 = (u128)a0 * b2 + (u128)a1 * b1 + (u128)a2 * b0 + (u128)a3 * b4_19 + (u128)a4 * b3_19;
  u128 c3 = (u128)a0 * b3 + (u128)a1 * b2 + (u128)a2 * b1 + (u128)a3 * b0 + (u128)a4 * b4_19;
  u128 c4 = (u128)a0 * b4 + (u128)a1 * b3 + (u128)a2 * b2 + (u128)a3 * b1 + (u128)a4 * b0;
  c1 += (uint64_t)(c0 >> 51); uint64_t r0 = (uint64_t)c0 & M51;
  c2 += (uint64_t)(c1 >> 51); uint64_t r1 = (uint64_t)c1 & M51;
  c3 += (uint64_t)(c2 >> 51); uint64_t r2 = (uint64_t)c2 & M51;
  c4 += (uint64_t)(c3 >> 51); uint64_t r3 = (uint64_t)c3 & M51;
  uint64_t carry = (uint64_t)(c4 >> 51); uint64_t r4 = (uint64_t)c4 & M51;
  r0 += carry * 19;
  r1 += r0 >> 51; r0 &= M51;
  r->v[0] = r0; r->v[1] = r1; r->v[2] = r2; r->v[3] = r3; r->v[4] = r4;
}
static void fe_sq(fe* r, const fe* a) {
  CNT_SQ;
  const uint64_t a0 = a->v[0], a1 = a->v[1], a2 = a->v[2], a3 = a->v[3], a4 = a->v[4];
  const uint64_t d0 = 2 * a0, d1 = 2 * a1, a3_19 = 19 * a3, a4_19 = 19 * a4;
  u128 c0 = (u128)a0 * a0 + (u128)d1 * a4_19 + (u128)(2 * a2) * a3_19;
  u128 c1 = (u128)d0 * a1 + (u128)(2 * a2) * a4_19 + (u128)a3 * a3_19;
  u128 c2 = (u128)d0 * a2 + (u128)a1 * a1 + (u128)(2 * a3) * a4_19;
  u128 c3 = (u128)d0 * a3 + (u128)d1 * a2 + (u128)a4 * a4_19;
  u128 c4 = (u128)d0 * a4 + (u128)d1 * a3 + (u128)a2 * a2;
  c1 += (uint64_t)(c0 >> 51); uint64_t r0 = (uint64_t)c0 & M51;
  c2 += (uint64_t)(c1 >> 51); uint64_t r1 = (uint64_t)c1 & M51;
  c3 += (uint64_t)(c2 >> 51); uint64_t r2 = (uint64_t)c2 & M51;
  c4 += (uint64_t)(c3 >> 51); uint64_t r3 = (uint64_t)c3 & M51;
  uint64_t carry = (uint64_t)(c4 >> 51); uint64_t r4 = (uint64_t)c4 & M51;
  r0 += carry * 19;
  r1 += r0 >> 51; r0 &= M51;
  r->v[0] = r0; r->v[1] = r1; r->v[2] = r2; r->v[3] = r3; r->v[4] = r4;
}
static void fe_sqn(fe* r, const fe* a, int n) {
  fe_sq(r, a);
  for (int i = 1; i < n; i++) fe_sq(r, r);
}
/* FieldElement51::from_bytes: 255 bits, top bit ignored, no reduction */
static void fe_frombytes(fe* r, const uint8_t* s) {
  uint64_t w[4];
  for (int i = 0; i < 4; i++) {
    w[i] = 0;
    for (int b = 7; b >= 0; b--) w[i] = (w[i] << 8) | s[8 * i + b];
  }
  r->v[0] = w[0] & M51;
  r->v[1] = ((w[0] >> 51) | (w[1] << 13)) & M51;
  r->v[2] = ((w[1] >> 38) | (w[2] << 26)) & M51;
  r->v[3] = ((w[2] >> 25) | (w[3] << 39)) & M51;
  r->v[4] = (w[3] >> 12) & M51;
}
/* canonical encoding (value mod p) */
static void fe_tobytes(uint8_t* s, const fe* a) {
  fe t = *a;
  fe_carry(&t);
  fe_carry(&t);
  /* now t < 2^255 + small; compute q = 1 iff t >= p */
  uint64_t q = (t.v[0] + 19) >> 51;
  q = (t.v[1] + q) >> 51;
  q = (t.v[2] + q) >> 51;
  q = (t.v[3] + q) >> 51;
  q = (t.v[4] + q) >> 51;
  t.v[0] += 19 * q;
  uint64_t c;
  c = t.v[0] >> 51; t.v[0] &= M51; t.v[1] += c;
  c = t.v[1] >> 51; t.v[1] &= M51; t.v[2] += c;
  c = t.v[2] >> 51; t.v[2] &= M51; t.v[3] += c;
  c = t.v[3] >> 51; t.v[3] &= M51; t.v[4] += c;
  t.v[4] &= M51;
  uint64_t w0 = t.v[0] | (t.v[1] << 51), w1 = (t.v[1] >> 13) | (t.v[2] << 38), w2 = (t.v[2] >> 26) | (t.v[3] << 25),
           w3 = (t.v[3] >> 39) | (t.v[4] << 12);
  uint64_t w[4] = {w0, w1, w2, w3};
  for (int i = 0; i < 4; i++)
    for (int b = 0; b < 8; b++) s[8 * i + b] = (uint8_t)(w[i] >> (8 * b));
}
static int fe_iszero(const fe* a) {
  uint8_t s[32];
  fe_tobytes(s, a);
  uint8_t o = 0;
  for (int i = 0; i < 32; i++) o |= s[i];
  return o == 0;
}
static int fe_eq(const fe* a, const fe* b) {
  uint8_t x[32], y[32];
  fe_tobytes(x, a);
  fe_tobytes(y, b);
  return memcmp(x, y, 32) == 0;
}
static int fe_isneg(const fe* a) {
  uint8_t s[32];
  fe_tobytes(s, a);
  return s[0] & 1;
}
static void fe_pow_chain(fe* z250, fe* z11, const fe* z) {
  fe z2, t, z9, z50, z100, z10, z20, z40, z5;
  fe_sq(&z2, z);
  fe_sqn(&t, &z2, 2);
  fe_mul(&z9, &t, z);
  fe_mul(z11, &z9, &z2);
  fe_sq(&t, z11);
  fe_mul(&z5, &t, &z9);
  fe_sqn(&t, &z5, 5);
  fe_mul(&z10, &t, &z5);
  fe_sqn(&t, &z10, 10);
  fe_mul(&z20, &t, &z10);
  fe_sqn(&t, &z20, 20);
  fe_mul(&z40, &t, &z20);
  fe_sqn(&t, &z40, 10);
  fe_mul(&z50, &t, &z10);
  fe_sqn(&t, &z50, 50);
  fe_mul(&z100, &t, &z50);
  fe_sqn(&t, &z100, 100);
  fe_mul(&t, &t, &z100);
  fe_sqn(&t, &t, 50);
  fe_mul(z250, &t, &z50);
}
static void fe_pow_p58(fe* r, const fe* z) {
  fe z250, z11, t;
  fe_pow_chain(&z250, &z11, z);
  fe_sqn(&t, &z250, 2);
  fe_mul(r, &t, z);
}
static void fe_invert(fe* r, const fe* z) {
  fe z250, z11, t;
  fe_pow_chain(&z250, &z11, z);
  fe_sqn(&t, &z250, 5);
  fe_mul(r, &t, &z11);
}

static fe FE_D, FE_D2, FE_SQRTM1;

/* =================================================================== group */
typedef struct { fe X, Y, Z, T; } ge3;       /* extended */
typedef struct { fe X, Y, Z; } ge2;          /* projective */
typedef struct { fe X, Y, Z, T; } ge1;       /* completed */
typedef struct { fe YpX, YmX, Z, T2d; } gec; /* ProjectiveNiels */
typedef struct { fe ypx, ymx, xy2d; } gen;   /* AffineNiels */

static void ge3_id(ge3* r) { fe_0(&r->X); fe_1(&r->Y); fe_1(&r->Z); fe_0(&r->T); }
static void ge2_id(ge2* r) { fe_0(&r->X); fe_1(&r->Y); fe_1(&r->Z); }
static void ge1_to2(ge2* r, const ge1* p) { fe_mul(&r->X, &p->X, &p->T); fe_mul(&r->Y, &p->Y, &p->Z); fe_mul(&r->Z, &p->Z, &p->T); }
static void ge1_to3(ge3* r, const ge1* p) {
  fe_mul(&r->X, &p->X, &p->T); fe_mul(&r->Y, &p->Y, &p->Z); fe_mul(&r->Z, &p->Z, &p->T); fe_mul(&r->T, &p->X, &p->Y);
}
static void ge3_to2(ge2* r, const ge3* p) { r->X = p->X; r->Y = p->Y; r->Z = p->Z; }
static void ge3_toc(gec* r, const ge3* p) {
  fe_add(&r->YpX, &p->Y, &p->X); fe_sub(&r->YmX, &p->Y, &p->X); r->Z = p->Z; fe_mul(&r->T2d, &p->T, &FE_D2);
}
static void ge2_dbl(ge1* r, const ge2* p) {
  fe xx, yy, b, a;
  fe_sq(&xx, &p->X); fe_sq(&yy, &p->Y); fe_sq(&b, &p->Z); fe_add(&b, &b, &b);
  fe_add(&a, &p->X, &p->Y); fe_sq(&a, &a);
  fe_add(&r->Y, &yy, &xx); fe_sub(&r->Z, &yy, &xx); fe_sub(&r->X, &a, &r->Y); fe_sub(&r->T, &b, &r->Z);
}
static void ge_addc(ge1* r, const ge3* p, const gec* q, int neg) {
  fe a, b, c, zz, ypx, ymx;
  fe_add(&ypx, &p->Y, &p->X); fe_sub(&ymx, &p->Y, &p->X);
  fe_mul(&b, &ypx, neg ? &q->YmX : &q->YpX);
  fe_mul(&a, &ymx, neg ? &q->YpX : &q->YmX);
  fe_mul(&c, &q->T2d, &p->T);
  fe_mul(&zz, &p->Z, &q->Z); fe_add(&zz, &zz, &zz);
  fe_sub(&r->X, &b, &a); fe_add(&r->Y, &b, &a);
  if (neg) { fe_sub(&r->Z, &zz, &c); fe_add(&r->T, &zz, &c); }
  else { fe_add(&r->Z, &zz, &c); fe_sub(&r->T, &zz, &c); }
}
static void ge_addn(ge1* r, const ge3* p, const gen* q, int neg) {
  fe a, b, c, zz, ypx, ymx;
  fe_add(&ypx, &p->Y, &p->X); fe_sub(&ymx, &p->Y, &p->X);
  fe_mul(&b, &ypx, neg ? &q->ymx : &q->ypx);
  fe_mul(&a, &ymx, neg ? &q->ypx : &q->ymx);
  fe_mul(&c, &q->xy2d, &p->T);
  fe_add(&zz, &p->Z, &p->Z);
  fe_sub(&r->X, &b, &a); fe_add(&r->Y, &b, &a);
  if (neg) { fe_sub(&r->Z, &zz, &c); fe_add(&r->T, &zz, &c); }
  else { fe_add(&r->Z, &zz, &c); fe_sub(&r->T, &zz, &c); }
}

/* curve25519-dalek FieldElement::sqrt_ratio_i */
static int fe_sqrt_ratio_i(fe* r, const fe* u, const fe* v) {
  fe v3, v7, t, check, nu, nui, ri;
  fe_sq(&v3, v); fe_mul(&v3, &v3, v);
  fe_sq(&v7, &v3); fe_mul(&v7, &v7, v);
  fe_mul(&t, u, &v7); fe_pow_p58(&t, &t);
  fe_mul(r, u, &v3); fe_mul(r, r, &t);
  fe_sq(&check, r); fe_mul(&check, &check, v);
  fe_neg(&nu, u); fe_mul(&nui, &nu, &FE_SQRTM1);
  int correct = fe_eq(&check, u), flipped = fe_eq(&check, &nu), flipped_i = fe_eq(&check, &nui);
  fe_mul(&ri, r, &FE_SQRTM1);
  if (flipped || flipped_i) *r = ri;
  if (fe_isneg(r)) fe_neg(r, r);
  return correct || flipped;
}

/* CompressedEdwardsY::decompress (dalek 3.x) */
static int ge_decompress(ge3* r, const uint8_t* s) {
  fe one, yy, u, v;
  fe_frombytes(&r->Y, s);
  fe_1(&one);
  fe_sq(&yy, &r->Y);
  fe_sub(&u, &yy, &one);
  fe_mul(&v, &yy, &FE_D); fe_add(&v, &v, &one);
  if (!fe_sqrt_ratio_i(&r->X, &u, &v)) return 0;
  if (s[31] >> 7) fe_neg(&r->X, &r->X);
  fe_1(&r->Z);
  fe_mul(&r->T, &r->X, &r->Y);
  return 1;
}

static int ge2_is_identity(const ge2* p) { return fe_iszero(&p->X) && fe_eq(&p->Y, &p->Z); }
static int ge3_is_small_order(const ge3* p) {
  ge2 q; ge1 t;
  ge3_to2(&q, p);
  for (int i = 0; i < 3; i++) { ge2_dbl(&t, &q); ge1_to2(&q, &t); }
  return ge2_is_identity(&q);
}
static int ge2_eq3(const ge2* p, const ge3* q) {
  fe a, b;
  fe_mul(&a, &p->X, &q->Z); fe_mul(&b, &q->X, &p->Z);
  if (!fe_eq(&a, &b)) return 0;
  fe_mul(&a, &p->Y, &q->Z); fe_mul(&b, &q->Y, &p->Z);
  return fe_eq(&a, &b);
}

/* ================================================================= scalars */
static const uint64_t SC_L[4] = {0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0, 0x1000000000000000ULL};
static const uint64_t SC_MU[5] = {0xed9ce5a30a2c131bULL, 0x2106215d086329a7ULL, 0xffffffffffffffebULL,
                                  0xffffffffffffffffULL, 0xfULL};

static void load_le64(uint64_t* w, const uint8_t* s, int nw) {
  for (int i = 0; i < nw; i++) {
    w[i] = 0;
    for (int b = 7; b >= 0; b--) w[i] = (w[i] << 8) | s[8 * i + b];
  }
}
static int sc_lt_l(const uint64_t* s) {
  for (int i = 3; i >= 0; i--) {
    if (s[i] < SC_L[i]) return 1;
    if (s[i] > SC_L[i]) return 0;
  }
  return 0;
}
/* x (8 limbs) mod l, Barrett with b = 2^64, k = 4 */
static void sc_reduce512(uint64_t* r, const uint64_t* x) {
  const uint64_t* q1 = x + 3; /* 5 limbs */
  uint64_t q2[10] = {0};
  for (int i = 0; i < 5; i++) {
    u128 c = 0;
    for (int j = 0; j < 5; j++) {
      c += (u128)q1[i] * SC_MU[j] + q2[i + j];
      q2[i + j] = (uint64_t)c;
      c >>= 64;
    }
    q2[i + 5] = (uint64_t)c;
  }
  const uint64_t* q3 = q2 + 5; /* 5 limbs */
  uint64_t r2[5] = {0};
  for (int i = 0; i < 5; i++) {
    u128 c = 0;
    for (int j = 0; i + j < 5 && j < 4; j++) {
      c += (u128)q3[i] * SC_L[j] + r2[i + j];
      r2[i + j] = (uint64_t)c;
      c >>= 64;
    }
    if (i + 4 < 5) r2[i + 4] += (uint64_t)c;
  }
  uint64_t t[5];
  u128 bw = 0;
  for (int i = 0; i < 5; i++) {
    u128 d = (u128)x[i] - r2[i] - bw;
    t[i] = (uint64_t)d;
    bw = (d >> 64) ? 1 : 0;
  }
  for (int rep = 0; rep < 3; rep++) {
    uint64_t u[5];
    u128 b2 = 0;
    for (int i = 0; i < 5; i++) {
      u128 d = (u128)t[i] - (i < 4 ? SC_L[i] : 0) - b2;
      u[i] = (uint64_t)d;
      b2 = (d >> 64) ? 1 : 0;
    }
    if (!b2) memcpy(t, u, sizeof t);
  }
  memcpy(r, t, 32);
}
static void sc_from_hash(uint64_t* r, const uint8_t h[64]) {
  uint64_t x[8];
  load_le64(x, h, 8);
  sc_reduce512(r, x);
}
static void sc_mul(uint64_t* r, const uint64_t* a, const uint64_t* b) {
  uint64_t x[8] = {0};
  for (int i = 0; i < 4; i++) {
    u128 c = 0;
    for (int j = 0; j < 4; j++) {
      c += (u128)a[i] * b[j] + x[i + j];
      x[i + j] = (uint64_t)c;
      c >>= 64;
    }
    x[i + 4] = (uint64_t)c;
  }
  sc_reduce512(r, x);
}
static void sc_add(uint64_t* r, const uint64_t* a, const uint64_t* b) {
  uint64_t x[8] = {0};
  u128 c = 0;
  for (int i = 0; i < 4; i++) {
    c += (u128)a[i] + b[i];
    x[i] = (uint64_t)c;
    c >>= 64;
  }
  x[4] = (uint64_t)c;
  sc_reduce512(r, x);
}
static void sc_neg(uint64_t* r, const uint64_t* a) {
  uint64_t z[4] = {0, 0, 0, 0};
  int isz = (a[0] | a[1] | a[2] | a[3]) == 0;
  u128 bw = 0;
  for (int i = 0; i < 4; i++) {
    u128 d = (u128)SC_L[i] - a[i] - bw;
    r[i] = (uint64_t)d;
    bw = (d >> 64) ? 1 : 0;
  }
  if (isz) memcpy(r, z, 32);
}

/* w-NAF of a scalar < 2^256: naf[0..257) digits, odd, |d| < 2^(w-1) */
static void wnaf(int8_t* naf, const uint64_t* s, int w) {
  uint64_t k[5] = {s[0], s[1], s[2], s[3], 0};
  memset(naf, 0, 257);
  const int64_t width = 1LL << w, half = width >> 1;
  for (int i = 0; i < 257; i++) {
    if (k[0] & 1) {
      int64_t d = (int64_t)(k[0] & (uint64_t)(width - 1));
      if (d >= half) d -= width;
      naf[i] = (int8_t)d;
      /* k -= d */
      if (d > 0) {
        u128 bw = 0;
        for (int j = 0; j < 5; j++) {
          u128 t = (u128)k[j] - (j == 0 ? (uint64_t)d : 0) - bw;
          k[j] = (uint64_t)t;
          bw = (t >> 64) ? 1 : 0;
        }
      } else {
        u128 c = (uint64_t)(-d);
        for (int j = 0; j < 5; j++) {
          c += k[j];
          k[j] = (uint64_t)c;
          c >>= 64;
        }
      }
    }
    for (int j = 0; j < 4; j++) k[j] = (k[j] >> 1) | (k[j + 1] << 63);
    k[4] >>= 1;
  }
}

/* odd multiples [1,3,...,127]B, AffineNiels (AFFINE_ODD_MULTIPLES_OF_BASEPOINT) */
static gen B_ODD[64];
static ge3 G_B;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void to_niels(gen* r, const ge3* p) {
  fe zi, x, y, xy;
  fe_invert(&zi, &p->Z);
  fe_mul(&x, &p->X, &zi); fe_mul(&y, &p->Y, &zi); fe_mul(&xy, &x, &y);
  fe_add(&r->ypx, &y, &x); fe_sub(&r->ymx, &y, &x); fe_mul(&r->xy2d, &xy, &FE_D2);
}

static void init_consts(void) {
  static const uint8_t d[32] = {0xa3, 0x78, 0x59, 0x13, 0xca, 0x4d, 0xeb, 0x75, 0xab, 0xd8, 0x41,
                                0x41, 0x4d, 0x0a, 0x70, 0x00, 0x98, 0xe8, 0x79, 0x77, 0x79, 0x40,
                                0xc7, 0x8c, 0x73, 0xfe, 0x6f, 0x2b, 0xee, 0x6c, 0x03, 0x52};
  static const uint8_t sqm1[32] = {0xb0, 0xa0, 0x0e, 0x4a, 0x27, 0x1b, 0xee, 0xc4, 0x78, 0xe4, 0x2f,
                                   0xad, 0x06, 0x18, 0x43, 0x2f, 0xa7, 0xd7, 0xfb, 0x3d, 0x99, 0x00,
                                   0x4d, 0x2b, 0x0b, 0xdf, 0xc1, 0x4f, 0x80, 0x24, 0x83, 0x2b};
  static const uint8_t by[32] = {0x58, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                                 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                                 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66};
  fe_frombytes(&FE_D, d);
  fe_add(&FE_D2, &FE_D, &FE_D);
  fe_frombytes(&FE_SQRTM1, sqm1);
  ge_decompress(&G_B, by);
  ge3 b2, cur;
  ge1 t;
  ge2 q;
  gec bc2;
  ge3_to2(&q, &G_B);
  ge2_dbl(&t, &q);
  ge1_to3(&b2, &t);
  ge3_toc(&bc2, &b2);
  cur = G_B;
  for (int i = 0; i < 64; i++) {
    to_niels(&B_ODD[i], &cur);
    ge_addc(&t, &cur, &bc2, 0);
    ge1_to3(&cur, &t);
  }
}
static void ensure_init(void) { pthread_once(&g_once, init_consts); }

/* vartime_double_scalar_mul_basepoint(a, A, b) = aA + bB */
static void double_scalar_mul(ge2* out, const uint64_t* a, const ge3* A, const uint64_t* b) {
  int8_t an[257], bn[257];
  wnaf(an, a, 5);
  wnaf(bn, b, 8);
  gec tabA[8]; /* A, 3A, ..., 15A */
  ge3 a2, cur;
  ge1 t;
  ge2 q;
  gec a2c;
  ge3_toc(&tabA[0], A);
  ge3_to2(&q, A);
  ge2_dbl(&t, &q);
  ge1_to3(&a2, &t);
  ge3_toc(&a2c, &a2);
  cur = *A;
  for (int i = 1; i < 8; i++) {
    ge_addc(&t, &cur, &a2c, 0);
    ge1_to3(&cur, &t);
    ge3_toc(&tabA[i], &cur);
  }
  int i = 256;
  while (i >= 0 && an[i] == 0 && bn[i] == 0) i--;
  ge2 r;
  ge2_id(&r);
  for (; i >= 0; i--) {
    ge2_dbl(&t, &r);
    if (an[i] || bn[i]) {
      ge3 e;
      if (an[i]) {
        ge1_to3(&e, &t);
        ge_addc(&t, &e, &tabA[(an[i] > 0 ? an[i] : -an[i]) / 2], an[i] < 0);
      }
      if (bn[i]) {
        ge1_to3(&e, &t);
        ge_addn(&t, &e, &B_ODD[(bn[i] > 0 ? bn[i] : -bn[i]) / 2], bn[i] < 0);
      }
    }
    ge1_to2(&r, &t);
  }
  *out = r;
}

/* Straus vartime multiscalar: sum s_i P_i (w-NAF 5 tables per point) */
static void straus(ge3* out, const uint64_t (*sc)[4], const ge3* pts, size_t n) {
  int8_t* nafs = (int8_t*)malloc(n * 257 + 1);
  gec* tabs = (gec*)malloc(sizeof(gec) * 8 * (n ? n : 1));
  for (size_t k = 0; k < n; k++) {
    wnaf(nafs + 257 * k, sc[k], 5);
    ge3 p2, cur;
    ge1 t;
    ge2 q;
    gec p2c;
    ge3_toc(&tabs[8 * k], &pts[k]);
    ge3_to2(&q, &pts[k]);
    ge2_dbl(&t, &q);
    ge1_to3(&p2, &t);
    ge3_toc(&p2c, &p2);
    cur = pts[k];
    for (int i = 1; i < 8; i++) {
      ge_addc(&t, &cur, &p2c, 0);
      ge1_to3(&cur, &t);
      ge3_toc(&tabs[8 * k + i], &cur);
    }
  }
  ge2 r;
  ge2_id(&r);
  ge1 t;
  for (int i = 256; i >= 0; i--) {
    ge2_dbl(&t, &r);
    for (size_t k = 0; k < n; k++) {
      int8_t d = nafs[257 * k + i];
      if (d) {
        ge3 e;
        ge1_to3(&e, &t);
        ge_addc(&t, &e, &tabs[8 * k + (d > 0 ? d : -d) / 2], d < 0);
      }
    }
    ge1_to2(&r, &t);
  }
  ge1 tt;
  /* to extended: X Z, Y Z, Z Z, X Y via completed form (X:Z, Y:T) with T = Z */
  tt.X = r.X; tt.Y = r.Y; tt.Z = r.Z; tt.T = r.Z;
  ge1_to3(out, &tt);
  free(nafs);
  free(tabs);
}

/* ============================================================ verification */
/* crypto::Signature::verify -> dalek 1.0.1 verify_strict.  0 = Ok, 1 = Err */
int coa_oracle_verify_strict(const uint8_t* msg, size_t msg_len, const uint8_t* pk, const uint8_t* sig) {
  ensure_init();
  uint64_t s[4];
  load_le64(s, sig + 32, 4);
  if ((sig[63] & 0xe0) || !sc_lt_l(s)) return 1;
  ge3 A, R;
  if (!ge_decompress(&A, pk)) return 1;
  if (!ge_decompress(&R, sig)) return 1;
  if (ge3_is_small_order(&R) || ge3_is_small_order(&A)) return 1;
  uint8_t h[64];
  sha512_ctx c;
  sha512_init(&c);
  sha512_update(&c, sig, 32);
  sha512_update(&c, pk, 32);
  sha512_update(&c, msg, msg_len);
  sha512_final(&c, h);
  uint64_t k[4];
  sc_from_hash(k, h);
  ge3 nA = A;
  fe_neg(&nA.X, &A.X);
  fe_neg(&nA.T, &A.T);
  ge2 Rp;
  double_scalar_mul(&Rp, k, &nA, s);
  return ge2_eq3(&Rp, &R) ? 0 : 1;
}

/* dalek 1.0.1 verify_batch with explicit 128-bit z_i (16 LE bytes each).
   All votes sign the same msg.  0 = Ok, 1 = Err. */
int coa_oracle_verify_batch(const uint8_t* msg, size_t msg_len, const uint8_t* pks, const uint8_t* sigs, size_t n,
                            const uint8_t* zs) {
  ensure_init();
  ge3* pts = (ge3*)malloc(sizeof(ge3) * (2 * n + 1));
  uint64_t(*scs)[4] = (uint64_t(*)[4])malloc(sizeof(uint64_t[4]) * (2 * n + 1));
  int rc = 1;
  uint64_t bcoef[4] = {0, 0, 0, 0};
  for (size_t i = 0; i < n; i++) { /* crypto loop: from_bytes(sig), decompress A */
    if (sigs[64 * i + 63] & 0xe0) goto out;
    if (!ge_decompress(&pts[1 + n + i], pks + 32 * i)) goto out;
  }
  for (size_t i = 0; i < n; i++) {
    uint64_t s[4], z[4] = {0, 0, 0, 0}, hr[4], t[4];
    load_le64(s, sigs + 64 * i + 32, 4);
    if (!sc_lt_l(s)) goto out;
    load_le64(z, zs + 16 * i, 2);
    uint8_t h[64];
    sha512_ctx c;
    sha512_init(&c);
    sha512_update(&c, sigs + 64 * i, 32);
    sha512_update(&c, pks + 32 * i, 32);
    sha512_update(&c, msg, msg_len);
    sha512_final(&c, h);
    sc_from_hash(hr, h);
    sc_mul(t, z, s);
    sc_add(bcoef, bcoef, t);
    memcpy(scs[1 + i], z, 32);
    sc_mul(scs[1 + n + i], z, hr);
  }
  for (size_t i = 0; i < n; i++)
    if (!ge_decompress(&pts[1 + i], sigs + 64 * i)) goto out;
  sc_neg(scs[0], bcoef);
  pts[0] = G_B;
  {
    ge3 sum;
    straus(&sum, (const uint64_t(*)[4])scs, pts, 2 * n + 1);
    ge2 q;
    ge3_to2(&q, &sum);
    rc = ge2_is_identity(&q) ? 0 : 1;
  }
out:
  free(pts);
  free(scs);
  return rc;
}

/* ---------------------------------------------------- multithreaded driver */
#define COA_ORACLE_MAX_THREADS 4096
typedef struct {
  const uint8_t *msgs, *pks, *sigs;
  size_t msg_len, lo, hi;
  uint8_t* out;
} job_t;

static void* verify_worker(void* p) {
  job_t* j = (job_t*)p;
  for (size_t i = j->lo; i < j->hi; i++)
    j->out[i] = (uint8_t)coa_oracle_verify_strict(j->msgs + i * j->msg_len, j->msg_len, j->pks + 32 * i,
                                                  j->sigs + 64 * i);
  return NULL;
}

void coa_oracle_verify_strict_many(const uint8_t* msgs, size_t msg_len, const uint8_t* pks, const uint8_t* sigs,
                                   size_t n, uint8_t* out, int nthreads) {
  ensure_init();
  if (nthreads < 1) nthreads = 1;
  if (nthreads > COA_ORACLE_MAX_THREADS) nthreads = COA_ORACLE_MAX_THREADS;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
  job_t* jobs = (job_t*)malloc(sizeof(job_t) * nthreads);
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = (job_t){msgs, pks, sigs, msg_len, n * t / nthreads, n * (t + 1) / nthreads, out};
    pthread_create(&th[t], NULL, verify_worker, &jobs[t]);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
}

/* ------------------------------------- Certificate::verify crypto, many
   Certificate::verify (primary/src/messages.rs:189-215) as the reference runs
   it, one certificate per call of the loop, with the three crypto checks
   evaluated independently (bit 1: SHA-512(header bytes)[..32] != id,
   messages.rs:49-51 / 70-84; bit 2: verify_strict(id, author, header sig),
   :64-66; bit 4: verify_batch(Certificate::digest, votes) with the given
   16-byte weights, :214 / 226-234).  Certificates are dealt to nthreads
   pthreads in contiguous ranges (CPU baseline: all host cores). */
typedef struct {
  const uint8_t *hdata, *ids, *origins, *hsigs, *vpks, *vsigs, *zs;
  const uint64_t *hoff, *rounds, *voff;
  size_t lo, hi;
  uint8_t* out;
} certjob_t;

static uint8_t cert_one(const certjob_t* j, size_t c) {
  uint8_t bits = 0, h[64], m[72];
  coa_oracle_sha512(j->hdata + j->hoff[c], j->hoff[c + 1] - j->hoff[c], h);
  if (memcmp(h, j->ids + 32 * c, 32) != 0) bits |= 1;
  if (coa_oracle_verify_strict(j->ids + 32 * c, 32, j->origins + 32 * c, j->hsigs + 64 * c)) bits |= 2;
  memcpy(m, j->ids + 32 * c, 32);
  for (int b = 0; b < 8; b++) m[32 + b] = (uint8_t)(j->rounds[c] >> (8 * b));
  memcpy(m + 40, j->origins + 32 * c, 32);
  coa_oracle_sha512(m, 72, h);
  const uint64_t v0 = j->voff[c], nv = j->voff[c + 1] - v0;
  if (coa_oracle_verify_batch(h, 32, j->vpks + 32 * v0, j->vsigs + 64 * v0, nv, j->zs + 16 * v0)) bits |= 4;
  return bits;
}

static void* cert_worker(void* p) {
  certjob_t* j = (certjob_t*)p;
  for (size_t c = j->lo; c < j->hi; c++) j->out[c] = cert_one(j, c);
  return NULL;
}

void coa_oracle_certificate_verify_many(const uint8_t* hdata, const uint64_t* hoff, const uint8_t* ids,
                                        const uint8_t* origins, const uint8_t* hsigs, const uint64_t* rounds,
                                        const uint8_t* vpks, const uint8_t* vsigs, const uint64_t* voff,
                                        const uint8_t* zs, size_t n, uint8_t* out, int nthreads) {
  ensure_init();
  if (nthreads < 1) nthreads = 1;
  if (nthreads > COA_ORACLE_MAX_THREADS) nthreads = COA_ORACLE_MAX_THREADS;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
  certjob_t* jobs = (certjob_t*)malloc(sizeof(certjob_t) * nthreads);
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = (certjob_t){hdata, ids, origins, hsigs, vpks, vsigs, zs, hoff, rounds, voff,
                          n * t / nthreads, n * (t + 1) / nthreads, out};
    pthread_create(&th[t], NULL, cert_worker, &jobs[t]);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
}

#ifdef COA_COUNT
void coa_oracle_counts(uint64_t* nmul, uint64_t* nsq) {
  *nmul = g_nmul;
  *nsq = g_nsq;
}
void coa_oracle_reset_counts(void) { g_nmul = g_nsq = 0; }
#endif

/* ------------------------------------------- SHA-512 multithreaded driver */
typedef struct {
  const uint8_t* data;
  const uint64_t* off;
  size_t lo, hi;
  uint8_t* out;
} shajob_t;

static void* sha_worker(void* p) {
  shajob_t* j = (shajob_t*)p;
  for (size_t i = j->lo; i < j->hi; i++) coa_oracle_sha512(j->data + j->off[i], j->off[i + 1] - j->off[i], j->out + 64 * i);
  return NULL;
}

void coa_oracle_sha512_many_mt(const uint8_t* data, const uint64_t* off, size_t n, uint8_t* out64, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > COA_ORACLE_MAX_THREADS) nthreads = COA_ORACLE_MAX_THREADS;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
  shajob_t* jobs = (shajob_t*)malloc(sizeof(shajob_t) * nthreads);
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = (shajob_t){data, off, n * t / nthreads, n * (t + 1) / nthreads, out64};
    pthread_create(&th[t], NULL, sha_worker, &jobs[t]);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
}
