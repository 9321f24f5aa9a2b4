// SHA-512 (FIPS 180-4) for gfx950: one message per lane, or per lane pair
// (round2 / compress_kw2: a round's two halves on two adjacent lanes).
//
// Replaces sha2 0.9 `Sha512` at the reference's digest sites
// (worker/src/processor.rs:38, primary/src/messages.rs:72-82,147-151,
// 228-232) and inside ed25519 verification (k = H(R || A || M),
// ed25519-dalek 1.0.1 verify_strict / verify_batch).
//
#pragma once
#include "coa_fe.h"

namespace coa_sha {

__device__ __constant__ static const uint64_t K512[80] = {
    0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull,
    0x3956c25bf348b538ull, 0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull,
    0xd807aa98a3030242ull, 0x12835b0145706fbeull, 0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull,
    0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull, 0xc19bf174cf692694ull,
    0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
    0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull,
    0x983e5152ee66dfabull, 0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull,
    0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull, 0x06ca6351e003826full, 0x142929670a0e6e70ull,
    0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull, 0x53380d139d95b3dfull,
    0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
    0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull,
    0xd192e819d6ef5218ull, 0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull,
    0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull, 0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull,
    0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull, 0x682e6ff3d6b2b8a3ull,
    0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
    0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull,
    0xca273eceea26619cull, 0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull,
    0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull, 0x113f9804bef90daeull, 0x1b710b35131c471bull,
    0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull, 0x431d67c49c100d4cull,
    0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull};

// 64-bit words live in VGPR pairs.  gfx950 has no 64-bit rotate, and hipcc
// lowers `(x >> n) | (x << (64 - n))` to two 64-bit shifts plus two ORs; a
// rotate is instead two v_alignbit_b32 (one per half), three-way XORs and
// Ch/Maj are one v_bitop3_b32 per half, and 64-bit adds are v_lshl_add_u64.
// That takes a round from ~75 to ~40 VALU instructions.
COA_DEV uint32_t lo32(uint64_t x) { return (uint32_t)x; }
COA_DEV uint32_t hi32(uint64_t x) { return (uint32_t)(x >> 32); }
// A register pair from two halves.  Built as a <2 x i32> bitcast, not as
// (hi << 32) | lo: LLVM splits an add of the shift/or form into a
// zero-extended low add, a separate high add and v_mov's of zero halves
// (~10 extra instructions per round); the bitcast keeps every 64-bit add a
// single v_lshl_add_u64 on a pair.
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
COA_DEV uint64_t mk64(uint32_t lo, uint32_t hi) {
  u32x2 v;
  v.x = lo;
  v.y = hi;
  return __builtin_bit_cast(uint64_t, v);
}

template <int N>
COA_DEV uint64_t rotr(uint64_t x) {
  static_assert(N > 0 && N < 64 && N != 32, "rotate amount");
  const uint32_t l = lo32(x), h = hi32(x);
  if constexpr (N < 32)
    return mk64(__builtin_amdgcn_alignbit(h, l, N), __builtin_amdgcn_alignbit(l, h, N));
  else
    return mk64(__builtin_amdgcn_alignbit(l, h, N - 32), __builtin_amdgcn_alignbit(h, l, N - 32));
}
template <int N>
COA_DEV uint64_t shr(uint64_t x) {
  static_assert(N > 0 && N < 32, "shift amount");
  return mk64(__builtin_amdgcn_alignbit(hi32(x), lo32(x), N), hi32(x) >> N);
}
// bitop3 truth tables over (S0, S1, S2) = (0xF0, 0xCC, 0xAA)
template <unsigned TT>
COA_DEV uint64_t bitop3(uint64_t a, uint64_t b, uint64_t c) {
  return mk64(__builtin_amdgcn_bitop3_b32(lo32(a), lo32(b), lo32(c), TT),
              __builtin_amdgcn_bitop3_b32(hi32(a), hi32(b), hi32(c), TT));
}
COA_DEV uint64_t xor3(uint64_t a, uint64_t b, uint64_t c) { return bitop3<0x96>(a, b, c); }
COA_DEV uint64_t ch(uint64_t e, uint64_t f, uint64_t g) { return bitop3<0xCA>(e, f, g); }
COA_DEV uint64_t maj(uint64_t a, uint64_t b, uint64_t c) { return bitop3<0xE8>(a, b, c); }

COA_DEV void init(uint64_t st[8]) {
  st[0] = 0x6a09e667f3bcc908ull;
  st[1] = 0xbb67ae8584caa73bull;
  st[2] = 0x3c6ef372fe94f82bull;
  st[3] = 0xa54ff53a5f1d36f1ull;
  st[4] = 0x510e527fade682d1ull;
  st[5] = 0x9b05688c2b3e6c1full;
  st[6] = 0x1f83d9abfb41bd6bull;
  st[7] = 0x5be0cd19137e2179ull;
}

// One round with the working variables passed by name (the usual renaming:
// only d and h are written).
COA_DEV void round_(uint64_t a, uint64_t b, uint64_t c, uint64_t& d, uint64_t e, uint64_t f, uint64_t g,
                    uint64_t& h, uint64_t kw) {
  const uint64_t t1 = h + xor3(rotr<14>(e), rotr<18>(e), rotr<41>(e)) + ch(e, f, g) + kw;
  const uint64_t t2 = xor3(rotr<28>(a), rotr<34>(a), rotr<39>(a)) + maj(a, b, c);
  d += t1;
  h = t1 + t2;
}

// One 128-byte block; W holds the 16 big-endian message words (clobbered).
// Five passes of 16 rounds: every W index is static (no dynamic VGPR
// indexing), K512 comes in through scalar loads.  Passes 2-5 first extend
// the schedule in place, W[i] = W[i] + s0(W[i+1]) + W[i+9] + s1(W[i+14])
// (indices mod 16), which is exactly W[t] from W[t-16], W[t-15], W[t-7] and
// W[t-2] when evaluated in increasing i.
COA_DEV void compress(uint64_t st[8], uint64_t W[16]) {
  uint64_t a = st[0], b = st[1], c = st[2], d = st[3];
  uint64_t e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll 1
  for (int r = 0; r < 80; r += 16) {
    if (r) {
#pragma unroll
      for (int i = 0; i < 16; i++) {
        const uint64_t w15 = W[(i + 1) & 15], w2 = W[(i + 14) & 15];
        W[i] += xor3(rotr<1>(w15), rotr<8>(w15), shr<7>(w15)) + W[(i + 9) & 15] +
                xor3(rotr<19>(w2), rotr<61>(w2), shr<6>(w2));
      }
    }
    const uint64_t* K = K512 + r;
    round_(a, b, c, d, e, f, g, h, K[0] + W[0]);
    round_(h, a, b, c, d, e, f, g, K[1] + W[1]);
    round_(g, h, a, b, c, d, e, f, K[2] + W[2]);
    round_(f, g, h, a, b, c, d, e, K[3] + W[3]);
    round_(e, f, g, h, a, b, c, d, K[4] + W[4]);
    round_(d, e, f, g, h, a, b, c, K[5] + W[5]);
    round_(c, d, e, f, g, h, a, b, K[6] + W[6]);
    round_(b, c, d, e, f, g, h, a, K[7] + W[7]);
    round_(a, b, c, d, e, f, g, h, K[8] + W[8]);
    round_(h, a, b, c, d, e, f, g, K[9] + W[9]);
    round_(g, h, a, b, c, d, e, f, K[10] + W[10]);
    round_(f, g, h, a, b, c, d, e, K[11] + W[11]);
    round_(e, f, g, h, a, b, c, d, K[12] + W[12]);
    round_(d, e, f, g, h, a, b, c, K[13] + W[13]);
    round_(c, d, e, f, g, h, a, b, K[14] + W[14]);
    round_(b, c, d, e, f, g, h, a, K[15] + W[15]);
  }
  st[0] += a;
  st[1] += b;
  st[2] += c;
  st[3] += d;
  st[4] += e;
  st[5] += f;
  st[6] += g;
  st[7] += h;
}

COA_DEV uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// Big-endian 64-bit message word from two little-endian dwords in memory order.
COA_DEV uint64_t be64(uint32_t lo_mem, uint32_t hi_mem) {
  return ((uint64_t)bswap32(lo_mem) << 32) | bswap32(hi_mem);
}

// Digest state -> the 64 output bytes viewed as 16 little-endian dwords
// (dword j = bytes 4j..4j+3), which is also the little-endian 512-bit integer
// Scalar::from_hash reduces.
COA_DEV void state_to_le_words(uint32_t out[16], const uint64_t st[8]) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    out[2 * i] = bswap32((uint32_t)(st[i] >> 32));
    out[2 * i + 1] = bswap32((uint32_t)st[i]);
  }
}

// ------------------------------------------------------------------------
// Messages that are the concatenation of up to three global-memory segments
// (R || A || M for k, prefix || M for signing).  When every segment length
// and pointer is a multiple of 4 (`aligned`, uniform per launch) words are
// gathered as dwords; otherwise byte by byte.
struct Segs {
  const uint8_t* p[3];
  uint32_t len[3];
};

COA_DEV uint32_t seg_byte(const Segs& s, uint32_t pos) {
  if (pos < s.len[0]) return s.p[0][pos];
  pos -= s.len[0];
  if (pos < s.len[1]) return s.p[1][pos];
  pos -= s.len[1];
  if (pos < s.len[2]) return s.p[2][pos];
  return 0;
}

// 4 message bytes at pos (pos % 4 == 0) as a little-endian dword, including
// the 0x80 terminator and zero padding (length words are added by the caller).
COA_DEV uint32_t seg_word(const Segs& s, uint32_t pos, uint32_t total, bool aligned) {
  if (pos + 4 <= total && aligned) {
    uint32_t q = pos;
    if (q < s.len[0]) return *(const uint32_t*)(s.p[0] + q);
    q -= s.len[0];
    if (q < s.len[1]) return *(const uint32_t*)(s.p[1] + q);
    q -= s.len[1];
    return *(const uint32_t*)(s.p[2] + q);
  }
  uint32_t w = 0;
#pragma unroll
  for (int b = 0; b < 4; b++) {
    const uint32_t q = pos + b;
    uint32_t byte = 0;
    if (q < total) byte = seg_byte(s, q);
    else if (q == total) byte = 0x80;
    w |= byte << (8 * b);
  }
  return w;
}

COA_DEV void hash_segs(uint64_t st[8], const Segs& s, bool aligned) {
  const uint32_t total = s.len[0] + s.len[1] + s.len[2];
  const uint32_t nblocks = (total + 17 + 127) / 128;
  init(st);
  for (uint32_t blk = 0; blk < nblocks; blk++) {
    uint64_t W[16];
    const uint32_t base = blk * 128;
#pragma unroll
    for (int w = 0; w < 16; w++) {
      const uint32_t lo = seg_word(s, base + 8 * w, total, aligned);
      const uint32_t hi = seg_word(s, base + 8 * w + 4, total, aligned);
      W[w] = be64(lo, hi);
    }
    if (blk == nblocks - 1) {
      W[14] = 0;  // message lengths here are < 2^61 bytes
      W[15] = (uint64_t)total * 8;
    }
    compress(st, W);
  }
}

// ------------------------------------------------------------------------
// SHA-512 of p[0 .. len) in global memory, one lane (the worker batch and
// header digests).  Every load is an aligned dword: a message that starts at
// byte m of a dword is realigned with v_alignbyte, so serialized headers at
// arbitrary offsets read 33 dwords per block instead of 128 bytes.  Dwords
// that hold a message byte stay inside that byte's page, so the up to three
// bytes read past the end never fault.  Block i+1's dwords are in flight
// while block i is compressed (a lone lane hashing a long header is
// latency-bound); the tail block(s) carry the 0x80 terminator and the
// 128-bit bit length.
COA_DEV uint32_t align_word(uint32_t lo, uint32_t hi, uint32_t m) {
  return __builtin_amdgcn_alignbyte(hi, lo, m);  // ({hi, lo} >> 8m)[31:0]
}

COA_DEV void hash_mem(uint64_t st[8], const uint8_t* p, uint64_t len) {
  init(st);
  const uint32_t m = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3);
  const uint32_t* b = reinterpret_cast<const uint32_t*>(p - m);  // dword holding p[0]
  uint64_t pos = 0;  // bytes hashed; b + pos / 4 holds p[pos]
  uint32_t nxt[33];
  if (len >= 128) {
#pragma unroll
    for (int q = 0; q < 32; q++) nxt[q] = b[q];
    nxt[32] = m ? b[32] : 0u;
  }
  for (; pos + 128 <= len; pos += 128) {
    uint64_t W[16];
#pragma unroll
    for (int w = 0; w < 16; w++)
      W[w] = be64(align_word(nxt[2 * w], nxt[2 * w + 1], m), align_word(nxt[2 * w + 1], nxt[2 * w + 2], m));
    if (pos + 256 <= len) {
      const uint32_t* nb = b + (pos + 128) / 4;
#pragma unroll
      for (int q = 0; q < 32; q++) nxt[q] = nb[q];
      nxt[32] = m ? nb[32] : 0u;
    }
    compress(st, W);
  }
  const uint32_t rem = (uint32_t)(len - pos);  // < 128 bytes left
  const uint32_t tail_blocks = rem + 17 <= 128 ? 1 : 2;
  const uint32_t* tb0 = b + pos / 4;
  for (uint32_t tb = 0; tb < tail_blocks; tb++) {
    uint32_t d[33];  // the dwords of this tail block that hold message bytes, else 0
#pragma unroll
    for (int q = 0; q < 33; q++) {
      const uint32_t at = tb * 32 + q;
      d[q] = 4 * at < m + rem ? tb0[at] : 0u;
    }
    uint64_t W[16];
#pragma unroll
    for (int w = 0; w < 16; w++) {
      uint32_t half[2];
#pragma unroll
      for (int hh = 0; hh < 2; hh++) {
        const int q = 2 * w + hh;
        uint32_t x = align_word(d[q], d[q + 1], m);
        // bytes at or after the end: 0, except 0x80 at offset rem
        const int k = (int)rem - (int)(tb * 128 + 4 * q);
        if (k <= 0) x = k == 0 ? 0x80u : 0u;
        else if (k < 4) x = (x & ((1u << (8 * k)) - 1u)) | (0x80u << (8 * k));
        half[hh] = x;
      }
      W[w] = be64(half[0], half[1]);
    }
    if (tb == tail_blocks - 1) {
      W[14] = len >> 61;
      W[15] = len << 3;
    }
    compress(st, W);
  }
}

// SHA-512 of a short message held in registers: NW little-endian dwords in
// memory order (4*NW <= 108 bytes, so one block).  Used for the certificate
// digest (72 B) and k = H(R || A || M) (96 B) inside the fused kernels.
template <int NW>
COA_DEV void hash_words(uint64_t st[8], const uint32_t* w) {
  static_assert(NW % 2 == 0 && 4 * NW + 17 <= 128, "one-block message");
  uint64_t W[16];
#pragma unroll
  for (int i = 0; i < 16; i++) {
    if (2 * i + 1 < NW) W[i] = be64(w[2 * i], w[2 * i + 1]);
    else if (2 * i == NW) W[i] = 0x8000000000000000ull;
    else W[i] = 0;
  }
  W[15] = (uint64_t)NW * 32;
  init(st);
  compress(st, W);
}

// ------------------------------------------------------------------------
// Latency path for ONE long message (a certificate's header digest): the
// message schedule does not depend on the chaining state, so lanes expand
// every block's W[0..79] + K[t] in parallel into LDS, and the hashing wave
// runs only the rounds (one LDS broadcast read per round instead of ~17
// schedule instructions).  A lone wave issues at most one instruction per
// ~4 cycles whatever the unit (the scalar unit measured slower: 9.5 us per
// block vs 8 us), so the instruction count of the serial stream is the
// latency.
COA_DEV uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// Block `blk` of the padded message p[0 .. len) (FIPS 180-4 padding; nblk
// blocks in total) as 16 big-endian words.
COA_DEV void padded_block(uint64_t W[16], const uint8_t* p, uint64_t len, uint64_t blk, uint64_t nblk) {
  const uint64_t base = blk * 128;
  if (base + 128 <= len && (reinterpret_cast<uintptr_t>(p) & 3) == 0) {
    const uint4* q = reinterpret_cast<const uint4*>(p + base);
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint4 v = q[i];
      W[2 * i] = be64(v.x, v.y);
      W[2 * i + 1] = be64(v.z, v.w);
    }
  } else {
#pragma unroll
    for (int w = 0; w < 16; w++) {
      uint32_t half[2];
#pragma unroll
      for (int hh = 0; hh < 2; hh++) {
        uint32_t x = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) {
          const uint64_t q = base + 8 * w + 4 * hh + b;
          uint32_t byte = 0;
          if (q < len) byte = p[q];
          else if (q == len) byte = 0x80;
          x |= byte << (8 * b);
        }
        half[hh] = x;
      }
      W[w] = be64(half[0], half[1]);
    }
  }
  if (blk == nblk - 1) {
    W[14] = len >> 61;
    W[15] = len << 3;
  }
}

// kw[t] = K[t] + W[t], t = 0..79, for one block.
COA_DEV void expand_kw(uint64_t* kw, uint64_t W[16]) {
#pragma unroll
  for (int i = 0; i < 16; i++) kw[i] = K512[i] + W[i];
#pragma unroll 1
  for (int r = 16; r < 80; r += 16) {
#pragma unroll
    for (int i = 0; i < 16; i++) {
      const uint64_t w15 = W[(i + 1) & 15], w2 = W[(i + 14) & 15];
      W[i] += xor3(rotr<1>(w15), rotr<8>(w15), shr<7>(w15)) + W[(i + 9) & 15] +
              xor3(rotr<19>(w2), rotr<61>(w2), shr<6>(w2));
      kw[r + i] = K512[r + i] + W[i];
    }
  }
}

// One block's 80 rounds from a precomputed kw (LDS, broadcast to the wave).
COA_DEV void compress_kw(uint64_t st[8], const uint64_t* kw) {
  uint64_t a = st[0], b = st[1], c = st[2], d = st[3];
  uint64_t e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll 1
  for (int r = 0; r < 80; r += 16) {
    const uint64_t* k = kw + r;
    round_(a, b, c, d, e, f, g, h, k[0]);
    round_(h, a, b, c, d, e, f, g, k[1]);
    round_(g, h, a, b, c, d, e, f, k[2]);
    round_(f, g, h, a, b, c, d, e, k[3]);
    round_(e, f, g, h, a, b, c, d, k[4]);
    round_(d, e, f, g, h, a, b, c, k[5]);
    round_(c, d, e, f, g, h, a, b, k[6]);
    round_(b, c, d, e, f, g, h, a, k[7]);
    round_(a, b, c, d, e, f, g, h, k[8]);
    round_(h, a, b, c, d, e, f, g, k[9]);
    round_(g, h, a, b, c, d, e, f, k[10]);
    round_(f, g, h, a, b, c, d, e, k[11]);
    round_(e, f, g, h, a, b, c, d, k[12]);
    round_(d, e, f, g, h, a, b, c, k[13]);
    round_(c, d, e, f, g, h, a, b, k[14]);
    round_(b, c, d, e, f, g, h, a, k[15]);
  }
  st[0] += a;
  st[1] += b;
  st[2] += c;
  st[3] += d;
  st[4] += e;
  st[5] += f;
  st[6] += g;
  st[7] += h;
}

// ------------------------------------------------------------------------
// One message on two lanes of a wave: the round's two halves in one
// instruction stream.  Even lanes hold (e, f, g, h) and compute
//   T1 = h + kw + S1(e) + Ch(e, f, g),
// odd lanes hold (a, b, c, d) and compute
//   T2 = S0(a) + Maj(a, b, c) = S0(a) + Ch(a ^ c, b, c),
// with per-lane operands only: both sums are r3-rotations of
// x ^ rotr(x, r1) ^ rotr(x, r2) (S1: 14 of 4 and 27; S0: 28 of 6 and 11, so
// every rotate is a pair of v_alignbit_b32 with a per-lane amount), Ch's first
// operand is x ^ (s2 & m) (m = 0 on even lanes), and h + kw is masked to 0 on
// odd lanes.  One DPP swap of adjacent lanes then hands the even lane d and
// the odd lane T1: the new e = d + T1 and the new a = T1 + T2 are both
// "received + own".  A lone wave issues one instruction per ~4 cycles, so
// single-message latency is the round's instruction count: ~22 here against
// ~28 for the one-lane round.
struct Lane2 {
  uint32_t r1, r2, r3, m, km;
  bool even;
};
COA_DEV Lane2 lane2(uint32_t lane) {
  Lane2 L;
  L.even = (lane & 1) == 0;
  L.r1 = L.even ? 4u : 6u;
  L.r2 = L.even ? 27u : 11u;
  L.r3 = L.even ? 14u : 28u;
  L.m = L.even ? 0u : ~0u;
  L.km = L.even ? ~0u : 0u;
  return L;
}
COA_DEV uint64_t rotr_v(uint64_t x, uint32_t n) {  // 0 < n < 32, per lane
  const uint32_t l = lo32(x), h = hi32(x);
  return mk64(__builtin_amdgcn_alignbit(h, l, n), __builtin_amdgcn_alignbit(l, h, n));
}
COA_DEV uint64_t swap_adjacent(uint64_t x) {  // lanes 2i <-> 2i + 1 (DPP quad_perm [1,0,3,2])
  return mk64((uint32_t)__builtin_amdgcn_mov_dpp((int)lo32(x), 0xB1, 0xF, 0xF, false),
              (uint32_t)__builtin_amdgcn_mov_dpp((int)hi32(x), 0xB1, 0xF, 0xF, false));
}
// (s0, s1, s2, s3) -> the lane's new s0, written into s3 (the caller renames).
COA_DEV void round2(uint64_t s0, uint64_t s1, uint64_t s2, uint64_t& s3, uint64_t kw, const Lane2& L) {
  const uint64_t in = xor3(s0, rotr_v(s0, L.r1), rotr_v(s0, L.r2));
  const uint64_t sg = rotr_v(in, L.r3);
  const uint64_t y = bitop3<0x78>(s0, s2, mk64(L.m, L.m));  // s0 ^ (s2 & m)
  const uint64_t t = sg + ch(y, s1, s2) + ((s3 + kw) & mk64(L.km, L.km));
  const uint64_t r = swap_adjacent(L.even ? t : s3);
  s3 = r + t;
}
// One block's 80 rounds on the lane's half state hs (even lanes: state words
// 4..7, odd lanes: 0..3) from a precomputed kw[t * STRIDE] (LDS; both lanes
// of a pair read the same word).  The words of the next 16 rounds are loaded
// while the current 16 run (two register sets, the 80 rounds unrolled): a
// lone wave has nothing else to cover an LDS round trip, and loading each
// group's words at its start left ~14 cycles of wait in every round (a C3
// header chain at 102 cycles a round against 88 for its 22 instructions,
// tools/cert_lat_probe.py).
template <int STRIDE>
COA_DEV void load16(uint64_t (&w)[16], const uint64_t* k) {
#pragma unroll
  for (int i = 0; i < 16; i++) w[i] = k[i * STRIDE];
}
COA_DEV void rounds16(uint64_t& a, uint64_t& b, uint64_t& c, uint64_t& d, const uint64_t (&w)[16], const Lane2& L) {
#pragma unroll
  for (int q = 0; q < 16; q += 4) {
    round2(a, b, c, d, w[q], L);
    round2(d, a, b, c, w[q + 1], L);
    round2(c, d, a, b, w[q + 2], L);
    round2(b, c, d, a, w[q + 3], L);
  }
}
template <int STRIDE = 1>
COA_DEV void compress_kw2(uint64_t hs[4], const uint64_t* kw, const Lane2& L) {
  uint64_t a = hs[0], b = hs[1], c = hs[2], d = hs[3];
  uint64_t w0[16], w1[16];
  load16<STRIDE>(w0, kw);
  load16<STRIDE>(w1, kw + 16 * STRIDE);
  rounds16(a, b, c, d, w0, L);  // rounds 0..15, 16..31 in flight
  load16<STRIDE>(w0, kw + 32 * STRIDE);
  rounds16(a, b, c, d, w1, L);
  load16<STRIDE>(w1, kw + 48 * STRIDE);
  rounds16(a, b, c, d, w0, L);
  load16<STRIDE>(w0, kw + 64 * STRIDE);
  rounds16(a, b, c, d, w1, L);
  rounds16(a, b, c, d, w0, L);
  hs[0] += a;
  hs[1] += b;
  hs[2] += c;
  hs[3] += d;
}
// The lane's half of the initial state / the full state on even lanes after
// the last block (odd partners hand over words 0..3).
COA_DEV void init2(uint64_t hs[4], const Lane2& L) {
  uint64_t st[8];
  init(st);
#pragma unroll
  for (int i = 0; i < 4; i++) hs[i] = L.even ? st[4 + i] : st[i];
}
COA_DEV void gather2(uint64_t st[8], const uint64_t hs[4]) {
#pragma unroll
  for (int i = 0; i < 4; i++) {
    st[i] = swap_adjacent(hs[i]);
    st[4 + i] = hs[i];
  }
}

// compress_kw with kw[t] at kw[t * STRIDE] (the shared-schedule kernel's
// lane-interleaved LDS layout).
template <int STRIDE>
COA_DEV void compress_kws(uint64_t st[8], const uint64_t* kw) {
  uint64_t a = st[0], b = st[1], c = st[2], d = st[3];
  uint64_t e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll 1
  for (int r = 0; r < 80; r += 16) {
    const uint64_t* k = kw + r * STRIDE;
    round_(a, b, c, d, e, f, g, h, k[0 * STRIDE]);
    round_(h, a, b, c, d, e, f, g, k[1 * STRIDE]);
    round_(g, h, a, b, c, d, e, f, k[2 * STRIDE]);
    round_(f, g, h, a, b, c, d, e, k[3 * STRIDE]);
    round_(e, f, g, h, a, b, c, d, k[4 * STRIDE]);
    round_(d, e, f, g, h, a, b, c, k[5 * STRIDE]);
    round_(c, d, e, f, g, h, a, b, k[6 * STRIDE]);
    round_(b, c, d, e, f, g, h, a, k[7 * STRIDE]);
    round_(a, b, c, d, e, f, g, h, k[8 * STRIDE]);
    round_(h, a, b, c, d, e, f, g, k[9 * STRIDE]);
    round_(g, h, a, b, c, d, e, f, k[10 * STRIDE]);
    round_(f, g, h, a, b, c, d, e, k[11 * STRIDE]);
    round_(e, f, g, h, a, b, c, d, k[12 * STRIDE]);
    round_(d, e, f, g, h, a, b, c, k[13 * STRIDE]);
    round_(c, d, e, f, g, h, a, b, k[14 * STRIDE]);
    round_(b, c, d, e, f, g, h, a, k[15 * STRIDE]);
  }
  st[0] += a;
  st[1] += b;
  st[2] += c;
  st[3] += d;
  st[4] += e;
  st[5] += f;
  st[6] += g;
  st[7] += h;
}

// expand_kw writing kw[t] to kw[t * STRIDE].
template <int STRIDE>
COA_DEV void expand_kws(uint64_t* kw, uint64_t W[16]) {
#pragma unroll
  for (int i = 0; i < 16; i++) kw[i * STRIDE] = K512[i] + W[i];
#pragma unroll 1
  for (int r = 16; r < 80; r += 16) {
#pragma unroll
    for (int i = 0; i < 16; i++) {
      const uint64_t w15 = W[(i + 1) & 15], w2 = W[(i + 14) & 15];
      W[i] += xor3(rotr<1>(w15), rotr<8>(w15), shr<7>(w15)) + W[(i + 9) & 15] +
              xor3(rotr<19>(w2), rotr<61>(w2), shr<6>(w2));
      kw[(r + i) * STRIDE] = K512[r + i] + W[i];
    }
  }
}

}  // namespace coa_sha
