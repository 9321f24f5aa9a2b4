// SHA-512 (FIPS 180-4) for gfx950, one message per lane.
//
// Replaces sha2 0.9 `Sha512` at the reference's digest sites
// (worker/src/processor.rs:38, primary/src/messages.rs:72-82,147-151,
// 228-232) and inside ed25519 verification (k = H(R || A || M),
// ed25519-dalek 1.0.1 verify_strict / verify_batch).
//
// 64-bit words are kept as uint64_t; hipcc lowers the rotations to
// v_alignbit_b32 pairs and Ch/Maj to v_bitop3_b32 on gfx950.
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

COA_DEV uint64_t rotr(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

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

// One 128-byte block; W holds the 16 big-endian message words (clobbered).
COA_DEV void compress(uint64_t st[8], uint64_t W[16]) {
  uint64_t a = st[0], b = st[1], c = st[2], d = st[3];
  uint64_t e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int t = 0; t < 80; t++) {
    uint64_t w;
    if (t < 16) {
      w = W[t];
    } else {
      const uint64_t w15 = W[(t - 15) & 15], w2 = W[(t - 2) & 15];
      const uint64_t s0 = rotr(w15, 1) ^ rotr(w15, 8) ^ (w15 >> 7);
      const uint64_t s1 = rotr(w2, 19) ^ rotr(w2, 61) ^ (w2 >> 6);
      w = W[t & 15] + s0 + W[(t - 7) & 15] + s1;
      W[t & 15] = w;
    }
    const uint64_t S1 = rotr(e, 14) ^ rotr(e, 18) ^ rotr(e, 41);
    const uint64_t ch = (e & f) ^ (~e & g);
    const uint64_t t1 = h + S1 + ch + K512[t] + w;
    const uint64_t S0 = rotr(a, 28) ^ rotr(a, 34) ^ rotr(a, 39);
    const uint64_t maj = (a & b) ^ (a & c) ^ (b & c);
    const uint64_t t2 = S0 + maj;
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
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

}  // namespace coa_sha
