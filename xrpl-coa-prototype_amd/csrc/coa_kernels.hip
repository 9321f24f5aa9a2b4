// Hand-written CDNA4 (gfx950) kernels for the ed25519 / SHA-512 verification
// engine.  One lane per signature (or per message); all arithmetic is integer
// VALU work (GF(2^255-19) and mod-l scalars), no MFMA.
//
// Reference behaviour replaced (see DESIGN.md for the full map):
//   k_hram            k = Scalar::from_hash(Sha512(R || A || M))
//                     (ed25519-dalek 1.0.1 verify_strict / verify_batch)
//   k_verify_strict   crypto::Signature::verify  (crypto/src/lib.rs:200-204)
//                     = ed25519::Signature::from_bytes + PublicKey::from_bytes
//                       + PublicKey::verify_strict
//   k_sha512_many     Sha512::digest(batch) (worker/src/processor.rs:38) and
//                     the Header/Vote/Certificate digests
//                     (primary/src/messages.rs:70-84,145-153,226-234)
//   k_keygen/k_sign_* RFC 8032 signing == crypto::Signature::new
//                     (crypto/src/lib.rs:185-191); used to synthesise inputs.
#include "coa_kernels.h"

#include <cstdlib>

#include "coa_fe.h"
#include "coa_ge.h"
#include "coa_sc.h"
#include "coa_sha512.h"
#include "coa_smul.h"

__global__ void __launch_bounds__(128) k_build_btable(uint32_t* tab) {
  const int j = threadIdx.x;  // multiple j+1
  ge_p3 B, acc;
  ge_basepoint(B);
  ge_cached Bc;
  ge_p3_to_cached(Bc, B);
  ge_p3_identity(acc);
  ge_p1p1 t;
  for (int bit = 7; bit >= 0; bit--) {
    ge_p3_dbl(t, acc);
    ge_p1p1_to_p3(acc, t);
    if (((j + 1) >> bit) & 1) {
      ge_add(t, acc, Bc);
      ge_p1p1_to_p3(acc, t);
    }
  }
  fe zi, x, y, xy, d2;
  fe_invert(zi, acc.Z);
  fe_mul(x, acc.X, zi);
  fe_mul(y, acc.Y, zi);
  fe_mul(xy, x, y);
  fe_const_d2(d2);
  fe n0, n1, n2;
  fe_add(n0, y, x);
  fe_sub(n1, y, x);
  fe_mul(n2, xy, d2);
  fe_canon(n0, n0);
  fe_canon(n1, n1);
  fe_canon(n2, n2);
  uint32_t* e = tab + j * 24;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    e[i] = n0.v[i];
    e[8 + i] = n1.v[i];
    e[16 + i] = n2.v[i];
  }
}


// ---------------------------------------------------------------------------
// k = SHA-512(R || A || M) mod l, one lane per signature.
// msg for signature i: msgs + (msg_index ? msg_index[i] : i) * msg_stride.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_hram(const uint8_t* __restrict__ msgs, uint32_t msg_len,
                                              uint64_t msg_stride, const uint32_t* __restrict__ msg_index,
                                              const uint8_t* __restrict__ pks, const uint8_t* __restrict__ sigs,
                                              uint32_t n, int aligned, uint32_t* __restrict__ k_out) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t mi = msg_index ? msg_index[i] : i;
    coa_sha::Segs s;
    s.p[0] = sigs + (uint64_t)i * 64;
    s.len[0] = 32;
    s.p[1] = pks + (uint64_t)i * 32;
    s.len[1] = 32;
    s.p[2] = msgs + mi * msg_stride;
    s.len[2] = msg_len;
    uint64_t st[8];
    coa_sha::hash_segs(st, s, aligned != 0);
    uint32_t h[16];
    coa_sha::state_to_le_words(h, st);
    sc k;
    sc_reduce512(k, h);
    uint4* o = reinterpret_cast<uint4*>(k_out + (uint64_t)i * 8);
    o[0] = make_uint4(k.v[0], k.v[1], k.v[2], k.v[3]);
    o[1] = make_uint4(k.v[4], k.v[5], k.v[6], k.v[7]);
  }
}

// ---------------------------------------------------------------------------
// Per-lane table of j·(-A), j = 1..8, in cached form: 8 entries x 32 dwords
// in a global scratch slab, lane-major: lane L's table is the 1 KiB at
// L * 1024 and entry e is the 128-byte line at + e * 128.  Lookups are
// data-dependent per lane, so this makes every lookup exactly one fully used
// cache line (an entry-major layout made each wave instruction touch up to 8
// rows: ~5x the fabric traffic, profiles/r01_v0_verify_traffic.json).
//   uint4 index = (lane * 8 + entry) * 8 + quad
// ---------------------------------------------------------------------------
COA_DEV void atab_store(uint32_t* __restrict__ scr, uint32_t lanes, uint32_t lane, int entry,
                        const ge_cached& q) {
  const fe* f[4] = {&q.YplusX, &q.YminusX, &q.Z, &q.T2d};
#pragma unroll
  for (int c = 0; c < 4; c++) {
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int quad = c * 2 + h;
      uint4* dst = reinterpret_cast<uint4*>(scr) + (((uint64_t)lane * 8 + entry) * 8 + quad);
      *dst = make_uint4(f[c]->v[4 * h], f[c]->v[4 * h + 1], f[c]->v[4 * h + 2], f[c]->v[4 * h + 3]);
    }
  }
}

COA_DEV void atab_select(ge_cached& q, const uint32_t* __restrict__ scr, uint32_t lanes, uint32_t lane,
                         int d) {
  const int m = d < 0 ? -d : d;
  const int entry = m == 0 ? 0 : m - 1;
  fe* f[4] = {&q.YplusX, &q.YminusX, &q.Z, &q.T2d};
#pragma unroll
  for (int c = 0; c < 4; c++) {
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int quad = c * 2 + h;
      const uint4 v = reinterpret_cast<const uint4*>(scr)[((uint64_t)lane * 8 + entry) * 8 + quad];
      f[c]->v[4 * h] = v.x;
      f[c]->v[4 * h + 1] = v.y;
      f[c]->v[4 * h + 2] = v.z;
      f[c]->v[4 * h + 3] = v.w;
    }
  }
  if (m == 0) ge_cached_identity(q);
  ge_cached_cneg(q, d < 0);
}

// R' = [k](-A) + [s]B by a joint Horner pass: 4 doublings per signed
// radix-16 digit of k, one cached addition of ±|d|·(-A), and every second
// digit one mixed addition of the signed radix-256 digit of s from the LDS
// B table.  Returns R' in projective form.
COA_DEV void double_scalar_mul(ge_p2& out, const uint32_t* kk, const uint32_t* ss, const uint32_t* scr,
                               uint32_t lanes, uint32_t lane, const uint32_t* btab) {
  uint32_t kp[8], sp[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    kp[i] = kk[i];
    sp[i] = ss[i];
  }
  add_const_word(kp, 0x88888888u);
  add_const_word(sp, 0x80808080u);
  ge_p3 acc3;
  ge_p2 acc2;
  ge_p1p1 t;
  ge_p3_identity(acc3);
#pragma unroll 1
  for (int i = 63; i >= 0; i--) {
    if (i != 63) {
#pragma unroll 1
      for (int dd = 0; dd < 3; dd++) {
        ge_p2_dbl(t, acc2);
        ge_p1p1_to_p2(acc2, t);
      }
      ge_p2_dbl(t, acc2);
      ge_p1p1_to_p3(acc3, t);
    }
    const int d = (int)take_top_bits(kp, 4) - 8;
    ge_cached qa;
    atab_select(qa, scr, lanes, lane, d);
    ge_add(t, acc3, qa);
    if ((i & 1) == 0) {
      const int e = (int)take_top_bits(sp, 8) - 128;
      ge_niels qb;
      btab_select(qb, btab, e);
      ge_p1p1_to_p3(acc3, t);
      ge_madd(t, acc3, qb);
    }
    ge_p1p1_to_p2(acc2, t);
  }
  out = acc2;
}

// ---------------------------------------------------------------------------
// crypto::Signature::verify == dalek 1.0.1 verify_strict, one lane per
// signature.  verdict 0 = Ok, 1 = Err.  k_in from k_hram.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256, 2) k_verify_strict(const uint8_t* __restrict__ pks,
                                                       const uint8_t* __restrict__ sigs,
                                                       const uint32_t* __restrict__ k_in, uint32_t n,
                                                       uint8_t* __restrict__ verdicts, uint32_t* __restrict__ scr,
                                                       const uint32_t* __restrict__ btab_g) {
  __shared__ __attribute__((aligned(16))) uint32_t btab[BTAB_DWORDS];
  lds_load_btable(btab, btab_g);
  const uint32_t lanes = gridDim.x * blockDim.x;
  const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
  for (uint32_t i = lane; i < n; i += lanes) {
    uint32_t aw[8], rw[8], sw[8], kw[8];
    {
      const uint4* p = reinterpret_cast<const uint4*>(pks + (uint64_t)i * 32);
      const uint4* g = reinterpret_cast<const uint4*>(sigs + (uint64_t)i * 64);
      const uint4* kq = reinterpret_cast<const uint4*>(k_in + (uint64_t)i * 8);
      uint4 v;
#define LD8(dst, src)                                                     \
  v = src[0];                                                             \
  dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; dst[3] = v.w;                 \
  v = src[1];                                                             \
  dst[4] = v.x; dst[5] = v.y; dst[6] = v.z; dst[7] = v.w;
      LD8(aw, p);
      LD8(rw, g);
      LD8(sw, (g + 2));
      LD8(kw, kq);
#undef LD8
    }
    // 1. s < l  (ed25519 1.x from_bytes + dalek check_scalar)
    bool ok = sc_is_canonical(sw);
    // 2./3. decompress A and R (dalek semantics), 4. neither small order
    ge_p3 A, R;
#pragma unroll 1
    for (int which = 0; which < 2; which++) {
      uint32_t w[8];
#pragma unroll
      for (int j = 0; j < 8; j++) w[j] = which ? rw[j] : aw[j];
      ge_p3 P;
      const bool dec = ge_decompress(P, w);
      const bool small = ge_is_small_order(P);
      ok = ok && dec && !small;
      if (which == 0) A = P;
      else R = P;
    }
    uint8_t verdict = 1;
    if (ok) {
      // table j·(-A), j = 1..8
      ge_p3 nA = A;
      fe_neg(nA.X, A.X);
      fe_neg(nA.T, A.T);
      ge_cached c1;
      ge_p3_to_cached(c1, nA);
      atab_store(scr, lanes, lane, 0, c1);
      ge_p3 cur = nA;
#pragma unroll 1
      for (int j = 1; j < 8; j++) {
        ge_p1p1 t;
        ge_add(t, cur, c1);
        ge_p1p1_to_p3(cur, t);
        ge_cached cj;
        ge_p3_to_cached(cj, cur);
        atab_store(scr, lanes, lane, j, cj);
      }
      // 6. [s]B + [k](-A) == R, compared projectively (cofactorless)
      ge_p2 Rp;
      double_scalar_mul(Rp, kw, sw, scr, lanes, lane, btab);
      verdict = ge_p2_eq_p3(Rp, R) ? 0 : 1;
    }
    verdicts[i] = verdict;
  }
}

// ---------------------------------------------------------------------------
// SHA-512 of n messages data[off[i] .. off[i+1]), one lane per message.
// out: 16 little-endian dwords (= the 64 digest bytes) per message.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_sha512_many(const uint8_t* __restrict__ data,
                                                     const uint64_t* __restrict__ off, uint32_t n,
                                                     uint32_t* __restrict__ out) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t o0 = off[i], o1 = off[i + 1];
    uint64_t st[8];
    coa_sha::hash_mem(st, data + o0, o1 - o0);
    uint32_t h[16];
    coa_sha::state_to_le_words(h, st);
    uint4* o = reinterpret_cast<uint4*>(out + (uint64_t)i * 16);
#pragma unroll
    for (int q = 0; q < 4; q++) o[q] = make_uint4(h[4 * q], h[4 * q + 1], h[4 * q + 2], h[4 * q + 3]);
  }
}

// ---------------------------------------------------------------------------
// SHA-512 of few long messages (worker batches): L lanes per message.  A lone
// lane hashing a 500 KB batch is bound by its own instruction stream (~42
// VALU instructions per round with the message schedule inline), and with
// fewer messages than 64 x SIMDs most of the chip idles.  Here the L lanes of
// a message expand the schedules of L consecutive blocks at once into LDS
// (kw[t][slot], slot = j * G + group, conflict-free), then all L run the
// rounds of those L blocks from LDS (28 instructions per round).  One
// 64-thread workgroup per wave; G = 64 / L messages per wave.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

template <int L, bool PF>
__global__ void __launch_bounds__(64) k_sha512_ml(const uint8_t* __restrict__ data, const uint64_t* __restrict__ off,
                                                  uint32_t n, uint32_t* __restrict__ out) {
  constexpr int G = 64 / L;
  __shared__ uint64_t kw[80 * 64];  // 40 KiB
  const uint32_t lane = threadIdx.x, grp = lane / L, q = lane % L;
  const uint32_t msg = blockIdx.x * G + grp;
  const bool live = msg < n;
  const uint64_t o0 = live ? off[msg] : 0, len = live ? off[msg + 1] - o0 : 0;
  const uint8_t* p = data + o0;
  const uint64_t nblk = live ? (len + 17 + 127) / 128 : 0;
  uint64_t maxblk = nblk;  // wave-uniform trip count
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t other = ((uint64_t)__shfl_xor((int)(maxblk >> 32), o, 64) << 32) |
                           (uint32_t)__shfl_xor((int)(uint32_t)maxblk, o, 64);
    maxblk = other > maxblk ? other : maxblk;
  }
  // the rounds on lane pairs (q even: state words 4..7, q odd: 0..3; L is
  // even, so a group's lanes pair up as 2i, 2i + 1): coa_sha512.h,
  // compress_kw2; lane q = 0 gathers the digest
  const coa_sha::Lane2 L2 = coa_sha::lane2(q);
  uint64_t hs[4];
  coa_sha::init2(hs, L2);
  // PF: the groups of blocks that are whole for every live message of the
  // wave run first, each lane's next block (b0 + L + q) loaded into
  // registers before the group's rounds run, so its global-memory latency
  // hides behind L compressions instead of sitting on the message's serial
  // chain (a lone wave per SIMD has no other wave to cover it); the padded
  // tail groups follow, loading on demand.  Kept as two loops: with the
  // padded loads in the same loop body the compiler's wait-count merge made
  // the wave wait for the prefetch (s_waitcnt vmcnt(0)) before its first
  // compression.
  // (dword loads: a message needs only 4-byte alignment -- C4's 508,052-byte
  // batches sit at 4-byte but not 16-byte offsets of the packed buffer)
  const uint64_t nwhole = (reinterpret_cast<uintptr_t>(p) & 3) == 0 ? len / 128 : 0;
  uint64_t fe = PF ? (live ? nwhole / L * L : ~0ull) : 0;  // wave-uniform end of the whole groups
#pragma unroll
  for (int o = 32; PF && o > 0; o >>= 1) {
    const uint64_t other = ((uint64_t)__shfl_xor((int)(fe >> 32), o, 64) << 32) |
                           (uint32_t)__shfl_xor((int)(uint32_t)fe, o, 64);
    fe = other < fe ? other : fe;
  }
  if (fe == ~0ull) fe = 0;
  uint64_t b0 = 0;
  if (PF && fe > 0) {
    // every lane loads and expands unconditionally (one straight-line body,
    // so the prefetch registers are not copied behind a wait): a live lane
    // its next whole block, clamped to its last one; a dead lane (no
    // message) re-reads the first block of `data`, which exists because a
    // live message of the wave has >= L whole blocks, and its state is never
    // written out
    const uint8_t* base = live ? p : data;
    const uint64_t last = live ? nwhole - 1 : 0;
    uint32_t nxt[32];
    {
      const uint32_t* src = reinterpret_cast<const uint32_t*>(base + (live ? (uint64_t)q : 0) * 128);
#pragma unroll
      for (int i = 0; i < 32; i++) nxt[i] = src[i];
    }
#pragma unroll 1
    for (; b0 < fe; b0 += L) {
      uint64_t W[16];
#pragma unroll
      for (int i = 0; i < 16; i++) W[i] = coa_sha::be64(nxt[2 * i], nxt[2 * i + 1]);
      const uint64_t nb = b0 + L + q < last ? b0 + L + q : last;
      const uint32_t* src = reinterpret_cast<const uint32_t*>(base + (live ? nb : 0) * 128);
#pragma unroll
      for (int i = 0; i < 32; i++) nxt[i] = src[i];
      coa_sha::expand_kws<64>(kw + q * G + grp, W);
      lds_sync();
#pragma unroll 1
      for (int j = 0; j < L; j++) coa_sha::compress_kw2<64>(hs, kw + j * G + grp, L2);
      lds_sync();
    }
  }
#pragma unroll 1
  for (; b0 < maxblk; b0 += L) {
    if (b0 + q < nblk) {
      uint64_t W[16];
      coa_sha::padded_block(W, p, len, b0 + q, nblk);
      coa_sha::expand_kws<64>(kw + q * G + grp, W);
    }
    __syncthreads();
#pragma unroll 1
    for (int j = 0; j < L; j++)
      if (b0 + j < nblk) coa_sha::compress_kw2<64>(hs, kw + j * G + grp, L2);
    __syncthreads();
  }
  uint64_t st[8];
  coa_sha::gather2(st, hs);
  if (live && q == 0) {
    uint32_t h[16];
    coa_sha::state_to_le_words(h, st);
    uint4* o = reinterpret_cast<uint4*>(out + (uint64_t)msg * 16);
#pragma unroll
    for (int i = 0; i < 4; i++) o[i] = make_uint4(h[4 * i], h[4 * i + 1], h[4 * i + 2], h[4 * i + 3]);
  }
}

// ---------------------------------------------------------------------------
// RFC 8032 signing (crypto::Signature::new / dalek Keypair::sign), used to
// synthesise benchmark inputs on the device.
// ---------------------------------------------------------------------------
// seeds (32 B each) -> public keys, expanded secret scalars a (mod l) and
// nonce prefixes.  aux layout per key: a (8 dwords) | prefix (8 dwords).
__global__ void __launch_bounds__(256) k_keygen(const uint8_t* __restrict__ seeds, uint32_t n,
                                                uint8_t* __restrict__ pks, uint32_t* __restrict__ aux,
                                                const uint32_t* __restrict__ btab_g) {
  __shared__ __attribute__((aligned(16))) uint32_t btab[BTAB_DWORDS];
  lds_load_btable(btab, btab_g);
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    coa_sha::Segs s;
    s.p[0] = seeds + (uint64_t)i * 32;
    s.len[0] = 32;
    s.p[1] = s.p[0];
    s.len[1] = 0;
    s.p[2] = s.p[0];
    s.len[2] = 0;
    uint64_t st[8];
    coa_sha::hash_segs(st, s, true);
    uint32_t h[16];
    coa_sha::state_to_le_words(h, st);
    h[0] &= ~7u;  // clamp
    h[7] &= 0x7fffffffu;
    h[7] |= 0x40000000u;
    uint32_t wide[16];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      wide[j] = h[j];
      wide[8 + j] = 0;
    }
    sc a;
    sc_reduce512(a, wide);
    ge_p2 P;
    fixed_base_mul(P, a.v, btab);
    uint32_t enc[8];
    ge_p2_compress(enc, P);
    uint4* pk = reinterpret_cast<uint4*>(pks + (uint64_t)i * 32);
    pk[0] = make_uint4(enc[0], enc[1], enc[2], enc[3]);
    pk[1] = make_uint4(enc[4], enc[5], enc[6], enc[7]);
    uint32_t* ax = aux + (uint64_t)i * 16;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      ax[j] = a.v[j];
      ax[8 + j] = h[8 + j];
    }
  }
}

// r = H(prefix || M) mod l; R = [r]B written to sigs[i][0..32); r kept in rbuf.
__global__ void __launch_bounds__(256) k_sign_r(const uint32_t* __restrict__ aux, const uint8_t* __restrict__ msgs,
                                                uint32_t msg_len, int aligned, uint32_t n,
                                                uint8_t* __restrict__ sigs, uint32_t* __restrict__ rbuf,
                                                const uint32_t* __restrict__ btab_g) {
  __shared__ __attribute__((aligned(16))) uint32_t btab[BTAB_DWORDS];
  lds_load_btable(btab, btab_g);
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    coa_sha::Segs s;
    s.p[0] = reinterpret_cast<const uint8_t*>(aux + (uint64_t)i * 16 + 8);
    s.len[0] = 32;
    s.p[1] = msgs + (uint64_t)i * msg_len;
    s.len[1] = msg_len;
    s.p[2] = s.p[1];
    s.len[2] = 0;
    uint64_t st[8];
    coa_sha::hash_segs(st, s, aligned != 0);
    uint32_t h[16];
    coa_sha::state_to_le_words(h, st);
    sc r;
    sc_reduce512(r, h);
    ge_p2 P;
    fixed_base_mul(P, r.v, btab);
    uint32_t enc[8];
    ge_p2_compress(enc, P);
    uint4* sg = reinterpret_cast<uint4*>(sigs + (uint64_t)i * 64);
    sg[0] = make_uint4(enc[0], enc[1], enc[2], enc[3]);
    sg[1] = make_uint4(enc[4], enc[5], enc[6], enc[7]);
    uint32_t* rr = rbuf + (uint64_t)i * 8;
#pragma unroll
    for (int j = 0; j < 8; j++) rr[j] = r.v[j];
  }
}

// S = r + k·a mod l written to sigs[i][32..64).
__global__ void __launch_bounds__(256) k_sign_s(const uint32_t* __restrict__ aux, const uint32_t* __restrict__ rbuf,
                                                const uint32_t* __restrict__ kbuf, uint32_t n,
                                                uint8_t* __restrict__ sigs) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    uint32_t a[8], r[8], k[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      a[j] = aux[(uint64_t)i * 16 + j];
      r[j] = rbuf[(uint64_t)i * 8 + j];
      k[j] = kbuf[(uint64_t)i * 8 + j];
    }
    sc S;
    sc_muladd(S, k, a, r);
    uint4* sg = reinterpret_cast<uint4*>(sigs + (uint64_t)i * 64 + 32);
    sg[0] = make_uint4(S.v[0], S.v[1], S.v[2], S.v[3]);
    sg[1] = make_uint4(S.v[4], S.v[5], S.v[6], S.v[7]);
  }
}

// ---------------------------------------------------------------------------
// Launch wrappers (host side, called by coa_runtime.cpp).
// ---------------------------------------------------------------------------
static inline uint32_t grid_for(uint64_t n, uint32_t block, uint32_t max_blocks) {
  uint64_t g = (n + block - 1) / block;
  if (g > max_blocks) g = max_blocks;
  if (g == 0) g = 1;
  return (uint32_t)g;
}

hipError_t coa_launch_build_btable(uint32_t* tab, hipStream_t s) {
  hipLaunchKernelGGL(k_build_btable, dim3(1), dim3(128), 0, s, tab);
  return hipGetLastError();
}

hipError_t coa_launch_hram(const uint8_t* msgs, uint32_t msg_len, uint64_t msg_stride, const uint32_t* msg_index,
                           const uint8_t* pks, const uint8_t* sigs, uint32_t n, uint32_t* k_out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const int aligned = ((msg_len & 3) == 0) && ((msg_stride & 3) == 0) && (((uintptr_t)msgs & 3) == 0);
  hipLaunchKernelGGL(k_hram, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, msgs, msg_len, msg_stride, msg_index,
                     pks, sigs, n, aligned, k_out);
  return hipGetLastError();
}

hipError_t coa_launch_verify_strict(const uint8_t* pks, const uint8_t* sigs, const uint32_t* k_in, uint32_t n,
                                    uint8_t* verdicts, uint32_t* scratch, uint32_t scratch_lanes,
                                    const uint32_t* btab, hipStream_t s) {
  if (n == 0) return hipSuccess;
  uint32_t blocks = grid_for(n, COA_VERIFY_BLOCK, scratch_lanes / COA_VERIFY_BLOCK);
  hipLaunchKernelGGL(k_verify_strict, dim3(blocks), dim3(COA_VERIFY_BLOCK), 0, s, pks, sigs, k_in, n, verdicts,
                     scratch, btab);
  return hipGetLastError();
}

hipError_t coa_launch_sha512_many(const uint8_t* data, const uint64_t* off, uint32_t n, uint32_t* out,
                                  hipStream_t s) {
  if (n == 0) return hipSuccess;
  // lanes per message: at least 1024 waves (one per SIMD; a message's
  // compressions are one serial chain, so a SIMD left without a wave is lost
  // time, and more lanes per message split its schedule work further) --
  // 16,384 worker batches take 4 lanes each (round 4 gave them 2: 512 waves,
  // half the SIMDs idle); COA_SHA_LANES overrides, COA_SHA_PREFETCH=0 turns
  // the next-block prefetch off (A/B; both read per call)
  uint32_t L = 1;
  while (L < 64 && (uint64_t)n * L < 65536) L *= 2;
  if (const char* e = getenv("COA_SHA_LANES")) L = (uint32_t)atoi(e);
  const char* pf_env = getenv("COA_SHA_PREFETCH");
  const bool pf = !(pf_env && pf_env[0] == '0');
  const uint32_t waves = (uint32_t)(((uint64_t)n * L + 63) / 64);
#define COA_SHA_ML(LL)                                                                                  \
  case LL:                                                                                              \
    if (pf)                                                                                             \
      hipLaunchKernelGGL((k_sha512_ml<LL, true>), dim3(waves), dim3(64), 0, s, data, off, n, out);   \
    else                                                                                                \
      hipLaunchKernelGGL((k_sha512_ml<LL, false>), dim3(waves), dim3(64), 0, s, data, off, n, out);  \
    break;
  switch (L) {
    COA_SHA_ML(2)
    COA_SHA_ML(4)
    COA_SHA_ML(8)
    COA_SHA_ML(16)
    COA_SHA_ML(32)
    COA_SHA_ML(64)
    default: hipLaunchKernelGGL(k_sha512_many, dim3(grid_for(n, 64, 65536)), dim3(64), 0, s, data, off, n, out);
  }
#undef COA_SHA_ML
  return hipGetLastError();
}

hipError_t coa_launch_keygen(const uint8_t* seeds, uint32_t n, uint8_t* pks, uint32_t* aux, const uint32_t* btab,
                             hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_keygen, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, seeds, n, pks, aux, btab);
  return hipGetLastError();
}

hipError_t coa_launch_sign_r(const uint32_t* aux, const uint8_t* msgs, uint32_t msg_len, uint32_t n, uint8_t* sigs,
                             uint32_t* rbuf, const uint32_t* btab, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const int aligned = ((msg_len & 3) == 0) && (((uintptr_t)msgs & 3) == 0);
  hipLaunchKernelGGL(k_sign_r, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, aux, msgs, msg_len, aligned, n, sigs,
                     rbuf, btab);
  return hipGetLastError();
}

hipError_t coa_launch_sign_s(const uint32_t* aux, const uint32_t* rbuf, const uint32_t* kbuf, uint32_t n,
                             uint8_t* sigs, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_sign_s, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, aux, rbuf, kbuf, n, sigs);
  return hipGetLastError();
}
