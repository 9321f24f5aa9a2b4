// Pippenger batch equation for gfx950: crypto::Signature::verify_batch
// (crypto/src/lib.rs:206-219) -> ed25519-dalek 1.0.1 verify_batch over ONE
// large group (dalek switches from Straus to Pippenger above 190 points;
// SURVEY.md §2 row 2).  Same equation and acceptance rules as coa_batch.hip:
//   Ok  iff  every s_i < l, every A_i and R_i decompresses, and
//            [-(sum z_i s_i mod l)]B + sum [z_i]R_i + sum [z_i h_i mod l]A_i == O
// computed exactly, so with the same z_i the verdict equals dalek's bit for
// bit (torsion components included) and equals the per-vote path's.
//
// Points (np = 2n + 1): R_0..R_{n-1}, A_0..A_{n-1}, B, affine Niels form
// (decompression yields Z = 1, so no inversion).  Scalars are recoded into
// signed radix-2^9 digits |d| <= 256: 15 windows for the 128-bit weights of
// R_i, 29 for the 253-bit scalars of A_i and B.
//
// Kernels:
//   k_msm_prep    two lanes per signature (A_i on one, R_i on the other):
//                 encoding checks, decompression to Niels form, z h mod l,
//                 digits, block partial sums of z s (288-bit integers)
//   k_msm_bpoint  one workgroup: b = -(sum z s) mod l, B and its digits
//   k_msm_bucket  one workgroup per (chunk of 256·run points, window) pair
//                 with points: LDS counting sort of the chunk's points by
//                 |digit|; every lane then adds `run` consecutive sorted
//                 points (balanced whatever the digit distribution),
//                 flushing each completed bucket segment; the segments of
//                 a bucket meet in a segmented scan over the lanes (LDS);
//                 large groups leave the 256 bucket sums for k_msm_bsum*,
//                 one chunk computes sum_j j·B_j by a 256-lane suffix scan
//                 plus a reduction (wave shuffles, LDS across the four waves)
//   k_msm_bsum1/2 bucket sums over the chunks, then sum_j j·B_j per window
//   k_msm_wsum    one workgroup per window: sum of the chunk partials
//   k_msm_final   one wave: Horner over the windows (9 doublings each) in
//                 row form (coa_fe_wave.h): each step's four products on the
//                 wave's four DPP rows at once, additions on the rows too;
//                 identity test, encoding flag -> verdict
#include "coa_msm.h"

#include <atomic>
#include <cstdlib>

#include "coa_fe.h"
#include "coa_ge.h"
#include "coa_ge_rows.h"
#include "coa_sc.h"

namespace {

constexpr int NB = COA_MSM_NB;
constexpr int WA = COA_MSM_WA;
constexpr int WR = COA_MSM_WR;
constexpr int MAXRUN = COA_MSM_RUN;
constexpr int CHUNK = COA_MSM_CHUNK;
// bucket segment slots per (chunk, window): 256 owners + 256 continuations
constexpr uint32_t SEG_SLOTS = 512;

// Digit rows (one per window) padded to whole 16-byte vectors, so the bucket
// kernel reads its chunk's digits with 16-byte loads.
__host__ __device__ inline uint32_t dig_stride(uint32_t np) { return (np + 7) & ~7u; }

// Signed radix-2^9 recoding of an 8-word little-endian scalar: W digits in
// [-256, 255] (a digit of value 256 never occurs: 511 + carry = 512 is 0
// with carry).  The scalars are < 2^253 (W = 29) or < 2^128 (W = 15), so
// the final carry is 0.
template <int W>
COA_DEV void recode(int* d, const uint32_t* x) {
  uint32_t carry = 0;
#pragma unroll
  for (int w = 0; w < W; w++) {
    const int b = 9 * w, k = b >> 5, s = b & 31;
    uint32_t v = x[k] >> s;
    if (s > 23 && k + 1 < 8) v |= x[k + 1] << (32 - s);
    v = (v & 511u) + carry;
    carry = v >= 256u ? 1u : 0u;
    d[w] = (int)v - (int)(carry << 9);
  }
}

COA_DEV void niels_store(uint32_t* dst, const ge_p3& p) {  // p affine (Z = 1)
  fe ypx, ymx, t2d, d2;
  fe_add(ypx, p.Y, p.X);
  fe_sub(ymx, p.Y, p.X);
  fe_const_d2(d2);
  fe_mul(t2d, p.T, d2);
  uint4* o = reinterpret_cast<uint4*>(dst);
  o[0] = make_uint4(ypx.v[0], ypx.v[1], ypx.v[2], ypx.v[3]);
  o[1] = make_uint4(ypx.v[4], ypx.v[5], ypx.v[6], ypx.v[7]);
  o[2] = make_uint4(ymx.v[0], ymx.v[1], ymx.v[2], ymx.v[3]);
  o[3] = make_uint4(ymx.v[4], ymx.v[5], ymx.v[6], ymx.v[7]);
  o[4] = make_uint4(t2d.v[0], t2d.v[1], t2d.v[2], t2d.v[3]);
  o[5] = make_uint4(t2d.v[4], t2d.v[5], t2d.v[6], t2d.v[7]);
}
COA_DEV void niels_load(ge_niels& q, const uint32_t* src) {
  const uint4* s = reinterpret_cast<const uint4*>(src);
  fe* f[3] = {&q.yplusx, &q.yminusx, &q.xy2d};
#pragma unroll
  for (int c = 0; c < 3; c++) {
    const uint4 a = s[2 * c], b = s[2 * c + 1];
    f[c]->v[0] = a.x;
    f[c]->v[1] = a.y;
    f[c]->v[2] = a.z;
    f[c]->v[3] = a.w;
    f[c]->v[4] = b.x;
    f[c]->v[5] = b.y;
    f[c]->v[6] = b.z;
    f[c]->v[7] = b.w;
  }
}

COA_DEV void p3_add(ge_p3& r, const ge_p3& a, const ge_p3& b) {
  ge_cached c;
  ge_p3_to_cached(c, b);
  ge_p1p1 t;
  ge_add(t, a, c);
  ge_p1p1_to_p3(r, t);
}

// LDS point arrays are word-major (word * slots + slot): lanes touching
// different slots hit different banks.
COA_DEV void lds_put(uint32_t* base, int slots, int slot, const ge_p3& p) {
  const fe* f[4] = {&p.X, &p.Y, &p.Z, &p.T};
#pragma unroll
  for (int c = 0; c < 4; c++)
#pragma unroll
    for (int i = 0; i < 8; i++) base[(c * 8 + i) * slots + slot] = f[c]->v[i];
}
COA_DEV void lds_get(ge_p3& p, const uint32_t* base, int slots, int slot) {
  fe* f[4] = {&p.X, &p.Y, &p.Z, &p.T};
#pragma unroll
  for (int c = 0; c < 4; c++)
#pragma unroll
    for (int i = 0; i < 8; i++) f[c]->v[i] = base[(c * 8 + i) * slots + slot];
}
COA_DEV void gbl_put(uint32_t* dst, const ge_p3& p) {
  const fe* f[4] = {&p.X, &p.Y, &p.Z, &p.T};
  uint4* o = reinterpret_cast<uint4*>(dst);
#pragma unroll
  for (int c = 0; c < 4; c++) {
    o[2 * c] = make_uint4(f[c]->v[0], f[c]->v[1], f[c]->v[2], f[c]->v[3]);
    o[2 * c + 1] = make_uint4(f[c]->v[4], f[c]->v[5], f[c]->v[6], f[c]->v[7]);
  }
}
COA_DEV void gbl_get(ge_p3& p, const uint32_t* src) {
  fe* f[4] = {&p.X, &p.Y, &p.Z, &p.T};
  const uint4* s = reinterpret_cast<const uint4*>(src);
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const uint4 a = s[2 * c], b = s[2 * c + 1];
    f[c]->v[0] = a.x;
    f[c]->v[1] = a.y;
    f[c]->v[2] = a.z;
    f[c]->v[3] = a.w;
    f[c]->v[4] = b.x;
    f[c]->v[5] = b.y;
    f[c]->v[6] = b.z;
    f[c]->v[7] = b.w;
  }
}
COA_DEV void p3_shfl_down(ge_p3& r, const ge_p3& p, int delta) {
  const fe* f[4] = {&p.X, &p.Y, &p.Z, &p.T};
  fe* g[4] = {&r.X, &r.Y, &r.Z, &r.T};
#pragma unroll
  for (int c = 0; c < 4; c++)
#pragma unroll
    for (int i = 0; i < 8; i++) g[c]->v[i] = __shfl_down(f[c]->v[i], delta, 64);
}
COA_DEV void p3_select(ge_p3& r, const ge_p3& a, bool c) {  // r = c ? a : r
  fe_cmov(r.X, a.X, c);
  fe_cmov(r.Y, a.Y, c);
  fe_cmov(r.Z, a.Z, c);
  fe_cmov(r.T, a.T, c);
}

// Block-wide sum of one point per lane (256 lanes); the result is valid in
// thread 0.  `tmp` holds 4 slots of LDS points.
COA_DEV void block_sum(ge_p3& acc, uint32_t* tmp) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
#pragma unroll 1
  for (int delta = 32; delta > 0; delta >>= 1) {
    ge_p3 q;
    p3_shfl_down(q, acc, delta);
    p3_add(acc, acc, q);
  }
  if (lane == 0) lds_put(tmp, 4, wave, acc);
  __syncthreads();
  if (t == 0) {
#pragma unroll 1
    for (int w = 1; w < 4; w++) {
      ge_p3 q;
      lds_get(q, tmp, 4, w);
      p3_add(acc, acc, q);
    }
  }
}

// sum_j j·B_j over a workgroup's 256 buckets, lane t holding B_{t+1}:
// S_t = sum_{t' >= t} B_{t'+1} by a suffix scan inside each wave plus the
// totals of the waves above, then a block sum; valid in thread 0.
COA_DEV void bucket_weighted_sum(ge_p3& S, uint32_t* s_tmp) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
#pragma unroll 1
  for (int delta = 1; delta < 64; delta <<= 1) {
    ge_p3 q, id;
    p3_shfl_down(q, S, delta);
    ge_p3_identity(id);
    p3_select(q, id, lane + delta >= 64);
    p3_add(S, S, q);
  }
  if (lane == 0) lds_put(s_tmp, 4, wave, S);  // wave totals
  __syncthreads();
#pragma unroll 1
  for (int k = wave + 1; k < 4; k++) {
    ge_p3 q;
    lds_get(q, s_tmp, 4, k);
    p3_add(S, S, q);
  }
  __syncthreads();
  block_sum(S, s_tmp);
}

}  // namespace

// ------------------------------------------------------------------ prep
// Rows: one 16-lane DPP row per point instead of one lane (small batches,
// where the decompression chain's latency is the whole kernel): the power
// chain runs on the row (coa_fe_wave.h), the row's lane 0 writes.
// Bound by the field products' issue (the decompressions' power chains):
// capping it at 128 VGPRs for four waves per SIMD instead of three, or
// sizing the grid to one resident round, left it at 4.2 ms for 2^22 points
// (profiles/r04_msm_ab.txt).
template <bool Rows>
__global__ void __launch_bounds__(256) k_msm_prep(const uint8_t* __restrict__ pks, const uint8_t* __restrict__ sigs,
                                                  const uint32_t* __restrict__ kbuf, const uint32_t* __restrict__ zs,
                                                  uint32_t n, uint32_t np, uint32_t* __restrict__ pts,
                                                  int16_t* __restrict__ dig, uint32_t* __restrict__ zpart,
                                                  uint32_t* __restrict__ bad, uint32_t ps) {
  __shared__ uint32_t red[9 * 256];
  uint32_t acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  constexpr uint32_t SH = Rows ? 4 : 0;
  const uint32_t stride = (gridDim.x * blockDim.x) >> SH;
  const bool leader = !Rows || (threadIdx.x & 15) == 0;
  // Two lanes (rows) per signature: 2i decompresses A_i and recodes z_i h_i,
  // 2i+1 decompresses R_i, checks s_i and recodes z_i.  The two
  // decompressions (the long dependent chains) run side by side, so a small
  // batch waits for one of them, not both.
  for (uint32_t j = (blockIdx.x * blockDim.x + threadIdx.x) >> SH; j < 2 * n; j += stride) {
    const uint32_t i = j >> 1;
    const bool is_r = (j & 1) != 0;
    uint32_t enc[8], z[8];
    const uint32_t* src = is_r ? reinterpret_cast<const uint32_t*>(sigs + (uint64_t)i * 64)
                               : reinterpret_cast<const uint32_t*>(pks + (uint64_t)i * 32);
#pragma unroll
    for (int w = 0; w < 8; w++) {
      enc[w] = src[w];
      z[w] = w < 4 ? zs[(uint64_t)i * 4 + w] : 0;
    }
    ge_p3 P;
    bool ok = ge_decompress<Rows>(P, enc);
    if (leader) niels_store(pts + (uint64_t)(is_r ? i : n + i) * ps, P);
    int d[WA];
    if (is_r) {
      uint32_t sw[8];
      const uint32_t* sg = reinterpret_cast<const uint32_t*>(sigs + (uint64_t)i * 64);
#pragma unroll
      for (int w = 0; w < 8; w++) sw[w] = sg[8 + w];
      ok = sc_is_canonical(sw) && ok;
      sc zsv;
      sc_mul(zsv, z, sw);
      if (!ok) {
#pragma unroll
        for (int w = 0; w < 8; w++) {
          z[w] = 0;
          zsv.v[w] = 0;
        }
      }
      recode<WR>(d, z);
      if (leader) {
#pragma unroll
        for (int w = 0; w < WR; w++) dig[(uint64_t)w * dig_stride(np) + i] = (int16_t)d[w];
        uint32_t cy = 0;
#pragma unroll
        for (int w = 0; w < 8; w++) acc[w] = addc32(acc[w], zsv.v[w], cy, cy);
        acc[8] += cy;
      }
    } else {
      uint32_t hw[8];
#pragma unroll
      for (int w = 0; w < 8; w++) hw[w] = kbuf[(uint64_t)i * 8 + w];
      sc a;
      sc_mul(a, z, hw);
      if (!ok) {
#pragma unroll
        for (int w = 0; w < 8; w++) a.v[w] = 0;
      }
      recode<WA>(d, a.v);
      if (leader) {
#pragma unroll
        for (int w = 0; w < WA; w++) dig[(uint64_t)w * dig_stride(np) + n + i] = (int16_t)d[w];
      }
    }
    if (!ok && leader) atomicOr(bad, 1u);
  }
  // block partial of sum z s (288-bit, no reduction)
  const int t = threadIdx.x;
#pragma unroll
  for (int j = 0; j < 9; j++) red[j * 256 + t] = acc[j];
  __syncthreads();
  for (int half = 128; half > 0; half >>= 1) {
    if (t < half) {
      uint32_t cy = 0;
#pragma unroll
      for (int j = 0; j < 9; j++) red[j * 256 + t] = addc32(red[j * 256 + t], red[j * 256 + t + half], cy, cy);
    }
    __syncthreads();
  }
  if (t < 9) zpart[blockIdx.x * 9 + t] = red[t * 256];
}

// ------------------------------------------------------------ B and -b
__global__ void __launch_bounds__(256) k_msm_bpoint(const uint32_t* __restrict__ zpart, uint32_t nparts, uint32_t n,
                                                    uint32_t np, uint32_t* __restrict__ pts,
                                                    int16_t* __restrict__ dig, uint32_t ps) {
  __shared__ uint32_t red[10 * 256];
  const int t = threadIdx.x;
  uint32_t acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (uint32_t p = t; p < nparts; p += 256) {
    uint32_t cy = 0;
#pragma unroll
    for (int j = 0; j < 9; j++) acc[j] = addc32(acc[j], zpart[p * 9 + j], cy, cy);
    acc[9] += cy;
  }
#pragma unroll
  for (int j = 0; j < 10; j++) red[j * 256 + t] = acc[j];
  __syncthreads();
  for (int half = 128; half > 0; half >>= 1) {
    if (t < half) {
      uint32_t cy = 0;
#pragma unroll
      for (int j = 0; j < 10; j++) red[j * 256 + t] = addc32(red[j * 256 + t], red[j * 256 + t + half], cy, cy);
    }
    __syncthreads();
  }
  if (t == 0) {
    uint32_t x[16];
#pragma unroll
    for (int j = 0; j < 16; j++) x[j] = j < 10 ? red[j * 256] : 0;
    sc b, nb;
    sc_reduce512(b, x);
    sc_neg(nb, b.v);
    ge_p3 B;
    ge_basepoint(B);
    niels_store(pts + (uint64_t)2 * n * ps, B);
    int d[WA];
    recode<WA>(d, nb.v);
#pragma unroll
    for (int w = 0; w < WA; w++) dig[(uint64_t)w * dig_stride(np) + 2 * n] = (int16_t)d[w];
  }
}

// ------------------------------------------------------- bucket phase
// Tree: the large-group form (bucket sums left for k_msm_bsum*), three
// workgroups per CU; else one chunk's sum_j j·B_j in the workgroup (small
// groups), two per CU (no spills).
template <bool Tree>
__global__ void __launch_bounds__(256, Tree ? 3 : 2) k_msm_bucket(const uint32_t* __restrict__ pts,
                                                       const int16_t* __restrict__ dig, uint32_t n, uint32_t np,
                                                       uint32_t run, uint32_t nchunks, uint32_t nrc,
                                                       uint32_t* __restrict__ segs, uint32_t* __restrict__ part,
                                                       uint32_t ps) {
  // 34 KiB of LDS and <= 168 VGPRs: three workgroups per CU.  The bucket segments go to this
  // (chunk, window)'s 64 KiB slice of `segs` (owner segments by bucket,
  // continuation segments by lane): written once, read once, L2-resident.
  __shared__ uint16_t s_sorted[CHUNK];     // (local << 1) | negative, grouped by |digit|
  __shared__ uint32_t s_tmp[32 * 4];       // wave totals / block sum
  __shared__ uint32_t s_hist[NB + 2];      // histogram, then scatter cursors
  __shared__ uint32_t s_off[NB + 2];       // s_off[j] = first sorted entry of bucket j
  __shared__ uint32_t s_wtot[4];

  // Only (chunk, window) pairs with points get a workgroup: the nrc chunks
  // of R points alone have WR windows (the weights z_i are 128-bit), the
  // others WA.  Logical block L runs over those pairs chunk by chunk.
  // XCD-aware order: consecutive hardware blocks go round-robin over the 8
  // XCDs, so hardware block h takes logical block (h % 8) * (G8 / 8) + h / 8:
  // every XCD gets the same number of pairs (a grid over all WA windows of
  // every chunk gave the XCDs holding R chunks half the work of the others)
  // and works through whole chunks, window after window (the chunk's points
  // stay in that XCD's L2).
  const uint32_t G = nrc * WR + (nchunks - nrc) * WA, per = gridDim.x >> 3;
  const uint32_t L = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (L >= G) return;
  const uint32_t ch = L < nrc * WR ? L / WR : nrc + (L - nrc * WR) / WA;
  const uint32_t w = L < nrc * WR ? L % WR : (L - nrc * WR) % WA;
  const uint32_t slot = ch * WA + w;  // segment slice of this (chunk, window)
  const uint32_t chunk = 256 * run;
  const uint32_t base = ch * chunk;
  const uint32_t cnt = min(chunk, np - base);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  uint32_t* out = part + ((uint64_t)w * nchunks + ch) * 32;
  const uint32_t rlo = (w >= WR && base < n) ? n - base : 0;  // skip R points above their windows
  // The chunk's digits, eight per 16-byte load, all loads in flight at once
  // and kept in registers for both passes of the counting sort (one load per
  // entry and pass, each waiting out its latency, took 1.45 ms of the 2^21
  // group's bucket phase).
  constexpr int VPT = CHUNK / 8 / 256;  // 16-byte vectors per thread
  const uint4* dv = reinterpret_cast<const uint4*>(dig + (uint64_t)w * dig_stride(np) + base);
  const uint32_t nvec = (cnt + 7) / 8;
  uint4 dgt[VPT];
#pragma unroll
  for (int k = 0; k < VPT; k++) {
    const uint32_t j = t + 256 * k;
    dgt[k] = j < nvec ? dv[j] : make_uint4(0, 0, 0, 0);
  }
  // digit q (0..7) of vector k, 0 outside [rlo, cnt)
  auto digit = [&](int k, int q) -> int {
    const uint32_t l = (t + 256 * k) * 8 + q;
    const uint32_t word = q < 2 ? dgt[k].x : q < 4 ? dgt[k].y : q < 6 ? dgt[k].z : dgt[k].w;
    const int d = (int16_t)(q & 1 ? word >> 16 : word & 0xffffu);
    return (l < cnt && l >= rlo) ? d : 0;
  };

  // the sort is a latency chain (loads, LDS atomics, barriers): at raised
  // priority beside the other workgroups' addition loops (-2.3 %)
  __builtin_amdgcn_s_setprio(2);
  for (int j = t; j < NB + 2; j += 256) s_hist[j] = 0;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < VPT; k++)
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int d = digit(k, q);
      if (d) atomicAdd(&s_hist[d < 0 ? -d : d], 1u);
    }
  __syncthreads();
  {  // exclusive scan of hist[1..256] (thread t: bucket t + 1)
    const uint32_t v = s_hist[t + 1];
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) s_wtot[wave] = x;
    __syncthreads();
    uint32_t pre = 0;
    for (int k = 0; k < wave; k++) pre += s_wtot[k];
    const uint32_t excl = pre + x - v;
    s_off[t + 1] = excl;
    if (t == 255) s_off[NB + 1] = pre + x;
    __syncthreads();
    s_hist[t + 1] = excl;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < VPT; k++)
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int d = digit(k, q);
      if (d) {
        const uint32_t l = (t + 256 * k) * 8 + q;
        const uint32_t pos = atomicAdd(&s_hist[d < 0 ? -d : d], 1u);
        s_sorted[pos] = (uint16_t)((l << 1) | (d < 0 ? 1u : 0u));
      }
    }
  __syncthreads();
  __builtin_amdgcn_s_setprio(0);
  const uint32_t nnz = s_off[NB + 1];

  // balanced accumulation: lane t adds sorted entries [t·run, (t+1)·run),
  // the load of the next point in flight during each addition (the points
  // are random 128-byte reads from the chunk's 2 MiB of points).  Iteration
  // e loads entry e and adds entry e - 1; no point is loaded before the loop:
  // with a load there, InstCombine folded the header's phi(load before the
  // loop, load in the loop) into one load of phi(addresses) at the top of
  // each iteration, consumed at once -- the prefetch gone, every addition
  // waiting out its miss (`s_waitcnt vmcnt(0)` ahead of each one in the
  // ISA).  Two independent chains per lane, and the products interleaved
  // column by column (ge_madd_il), were no faster (profiles/r04_msm_ab.txt).
  uint32_t* const seg = segs + (uint64_t)slot * SEG_SLOTS * 32;  // [bucket - 1] owners, [256 + lane] continuations
  {
    const uint32_t lo = t * run, hi = min(lo + run, nnz);
    if (lo < hi) {
      const uint32_t* pb = pts + (uint64_t)base * ps;
      uint32_t cur = 1;  // bucket of entry lo: last j with s_off[j] <= lo
#pragma unroll
      for (uint32_t step = 128; step > 0; step >>= 1)
        if (s_off[cur + step] <= lo) cur += step;
      bool owner = s_off[cur] == lo;
      uint32_t nxt = s_off[cur + 1];
      ge_niels q;
      ge_niels_identity(q);
      uint32_t ent = 0;
      ge_p3 acc;
      ge_p3_identity(acc);
#pragma unroll 1
      for (uint32_t e = lo; e <= hi; e++) {
        ge_niels qn;
        uint32_t entn = 0;
        if (e < hi) {
          entn = s_sorted[e];
          niels_load(qn, pb + (uint64_t)(entn >> 1) * ps);
        } else {
          ge_niels_identity(qn);
        }
        if (e > lo) {  // add entry e - 1 (e - lo is the same on every lane)
          if (e - 1 == nxt) {  // bucket cur is complete: flush, move to the bucket of e - 1
            gbl_put(seg + (owner ? cur - 1 : 256 + t) * 32, acc);
            ge_p3_identity(acc);
            owner = true;
            do {
              cur++;
              nxt = s_off[cur + 1];
            } while (nxt == e - 1);
          }
          ge_niels_cneg(q, (ent & 1u) != 0);
          ge_p1p1 r;
          ge_madd(r, acc, q);
          ge_p1p1_to_p3(acc, r);
        }
        q = qn;
        ent = entn;
      }
      gbl_put(seg + (owner ? cur - 1 : 256 + t) * 32, acc);
    }
  }

  // Merge: bucket b's sum is its owner segment plus the continuation
  // segments ("pieces") of the lanes whose runs start strictly inside it,
  // lanes f_b .. g_b (contiguous).  Pieces are summed by a segmented
  // Hillis-Steele scan over the 256 lanes in LDS (the sorted entries' 32 KiB,
  // free now), ceil(log2(longest piece list)) rounds, so a bucket holding
  // most of the chunk -- the top window's digits (z_i < 2^128: |d| <= 4;
  // z h mod l < 2^253: |d| <= 1), or equal weights -- costs ~8 dependent
  // additions instead of one lane adding up to 255 pieces in a row (that
  // chain, in the top windows' workgroups, was 0.76 ms of the 2^21 group's
  // bucket phase: profiles/r04_msm_ab.txt).
  __syncthreads();  // every flush is out; s_sorted is free
  uint32_t* const s_pc = reinterpret_cast<uint32_t*>(s_sorted);  // [32 words][256 lanes]
  static_assert(CHUNK * 2 >= 256 * 128, "piece scratch");
  ge_p3 C;
  ge_p3_identity(C);
  uint32_t pf = t + 1;  // first piece lane of this lane's bucket (t + 1: no piece)
  {
    const uint32_t e = t * run;
    if (e < nnz) {
      uint32_t b = 1;
#pragma unroll
      for (uint32_t step = 128; step > 0; step >>= 1)
        if (s_off[b + step] <= e) b += step;
      if (s_off[b] != e) {  // this lane's run starts inside bucket b: a piece
        pf = s_off[b] / run + 1;
        gbl_get(C, seg + (256 + t) * 32);
      }
    }
  }
  uint32_t len = t + 1 - pf;  // this lane's position in its piece list (0: none)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) len = max(len, (uint32_t)__shfl_xor((int)len, o, 64));
  if ((t & 63) == 0) s_wtot[wave] = len;
  __syncthreads();
  const uint32_t maxlen = max(max(s_wtot[0], s_wtot[1]), max(s_wtot[2], s_wtot[3]));
#pragma unroll 1
  for (uint32_t st = 1; st < maxlen; st <<= 1) {
    lds_put(s_pc, 256, t, C);
    __syncthreads();
    if (t >= pf + st && t < 256) {  // t - st is a piece of the same bucket
      ge_p3 h;
      lds_get(h, s_pc, 256, t - st);
      p3_add(C, C, h);
    }
    __syncthreads();
  }
  lds_put(s_pc, 256, t, C);  // lane g_b now holds the sum of bucket b's pieces
  __syncthreads();
  // lane t: bucket t + 1 = owner segment + its pieces' sum (lane g)
  ge_p3 S;
  ge_p3_identity(S);
  {
    const uint32_t o0 = s_off[t + 1], o1 = s_off[t + 2];
    if (o1 > o0) {
      gbl_get(S, seg + t * 32);
      const uint32_t f = o0 / run + 1, g = (o1 - 1) / run;
      if (g >= f) {
        ge_p3 h;
        lds_get(h, s_pc, 256, g);
        p3_add(S, S, h);
      }
    }
  }
  if constexpr (Tree) {  // bucket sums of this (chunk, window) to its owner slots; summed over chunks by k_msm_bsum*
    gbl_put(seg + t * 32, S);
    return;
  }
  // sum_j j·B_j = sum_t S_t with S_t = sum_{t' >= t} B_{t'+1}
  bucket_weighted_sum(S, s_tmp);
  if (t == 0) gbl_put(out, S);
}

// Tree form of the window sums (COA_MSM_TREE): the bucket workgroups leave
// each (chunk, window)'s 256 bucket sums in their owner slots instead of
// running sum_j j·B_j per chunk (a 256-lane suffix scan and a block sum, ~20
// extended additions on every lane of every one of the 29 x nchunks
// workgroups); the buckets are summed over the chunks first -- one addition
// per (chunk, window, bucket) -- and the weighted sum runs once per window.
// Level 1: workgroup (window w, group g) adds bucket t over chunks
// [16g, 16g + 16) into the slot of chunk 16g.  (One wave per (window,
// bucket) with a 64-lane shuffle tree instead -- a 10-addition chain against
// 33 -- took 196 us against 105: twenty times the additions, at three waves
// per SIMD, made it throughput-bound.)
constexpr uint32_t kTreeGroup = 16;
// The nrc chunks of R points alone have no workgroup (and no segments) in
// windows >= WR: their buckets are empty there and are skipped.
__global__ void __launch_bounds__(256) k_msm_bsum1(uint32_t* __restrict__ segs, uint32_t nchunks, uint32_t nrc) {
  const uint32_t groups = (nchunks + kTreeGroup - 1) / kTreeGroup;
  const uint32_t w = blockIdx.x / groups, g = blockIdx.x % groups;
  const uint32_t t = threadIdx.x;
  const uint32_t c0 = g * kTreeGroup, c1 = min(nchunks, c0 + kTreeGroup);
  const uint32_t first = w >= WR ? max(c0, nrc) : c0;
  ge_p3 acc;
  if (first < c1)
    gbl_get(acc, segs + (((uint64_t)first * WA + w) * SEG_SLOTS + t) * 32);
  else
    ge_p3_identity(acc);
#pragma unroll 1
  for (uint32_t c = first + 1; c < c1; c++) {
    ge_p3 q;
    gbl_get(q, segs + (((uint64_t)c * WA + w) * SEG_SLOTS + t) * 32);
    p3_add(acc, acc, q);
  }
  gbl_put(segs + (((uint64_t)c0 * WA + w) * SEG_SLOTS + t) * 32, acc);
}
// Level 2: one workgroup per window: bucket t over the groups, then
// sum_j j·B_j once -> wsum (the layout k_msm_wsum writes).
__global__ void __launch_bounds__(256) k_msm_bsum2(const uint32_t* __restrict__ segs, uint32_t nchunks,
                                                   uint32_t* __restrict__ wsum) {
  __shared__ uint32_t s_tmp[32 * 4];
  const uint32_t w = blockIdx.x, t = threadIdx.x;
  ge_p3 S;
  gbl_get(S, segs + (((uint64_t)0 * WA + w) * SEG_SLOTS + t) * 32);
#pragma unroll 1
  for (uint32_t c = kTreeGroup; c < nchunks; c += kTreeGroup) {
    ge_p3 q;
    gbl_get(q, segs + (((uint64_t)c * WA + w) * SEG_SLOTS + t) * 32);
    p3_add(S, S, q);
  }
  bucket_weighted_sum(S, s_tmp);
  if (t == 0) gbl_put(wsum + (uint64_t)w * 32, S);
}

// ----------------------------------------------------------- window sums
__global__ void __launch_bounds__(256) k_msm_wsum(const uint32_t* __restrict__ part, uint32_t nchunks, uint32_t nrc,
                                                  uint32_t* __restrict__ wsum) {
  __shared__ uint32_t tmp[32 * 4];
  const uint32_t w = blockIdx.x;
  ge_p3 acc;
  ge_p3_identity(acc);
  for (uint32_t c = threadIdx.x + (w >= WR ? nrc : 0); c < nchunks; c += 256) {
    ge_p3 q;
    gbl_get(q, part + ((uint64_t)w * nchunks + c) * 32);
    p3_add(acc, acc, q);
  }
  block_sum(acc, tmp);
  if (threadIdx.x == 0) gbl_put(wsum + (uint64_t)w * 32, acc);
}

// ------------------------------------------------------ Horner + verdict

__global__ void __launch_bounds__(64) k_msm_final(const uint32_t* __restrict__ wsum, const uint32_t* __restrict__ bad,
                                                  uint8_t* __restrict__ verdict) {
  __shared__ uint32_t cw[WA * 32];  // cached form of every window sum
  const int t = threadIdx.x;
  if (t < WA) {
    ge_p3 p;
    gbl_get(p, wsum + (uint64_t)t * 32);
    ge_cached c;
    ge_p3_to_cached(c, p);
    const fe* f[4] = {&c.YplusX, &c.YminusX, &c.Z, &c.T2d};
#pragma unroll
    for (int q = 0; q < 4; q++)
#pragma unroll
      for (int i = 0; i < 8; i++) cw[t * 32 + q * 8 + i] = f[q]->v[i];
  }
  __syncthreads();
  const uint32_t* top = wsum + (uint64_t)(WA - 1) * 32;
  rp::P2 acc = {rp::ld(top), rp::ld(top + 8), rp::ld(top + 16)};
  rp::L1 r;
  rp::P1 a3;
#pragma unroll 1
  for (int w = WA - 2; w >= 0; w--) {
#pragma unroll 1
    for (int j = 0; j < COA_MSM_C - 1; j++) {
      rp::dbl(r, acc);
      rp::to_p2(acc, r);
    }
    rp::dbl(r, acc);
    rp::to_p3(a3, r);
    const uint32_t* q = cw + w * 32;
    const rp::Ca c = {rp::ld(q), rp::ld(q + 8), rp::ld(q + 16), rp::ld(q + 24)};
    rp::add(r, a3, c);
    rp::to_p2(acc, r);
  }
  ge_p2 res;
  fw::to_fe(res.X, acc.X);
  fw::to_fe(res.Y, acc.Y);
  fw::to_fe(res.Z, acc.Z);
  if (t == 0) verdict[0] = (ge_p2_is_identity(res) && bad[0] == 0) ? 0 : 1;
}

// ----------------------------------------------------------------- host
uint32_t coa_msm_chunks_run(size_t n, uint32_t run) {
  const size_t np = 2 * n + 1, chunk = 256 * (size_t)run;
  return (uint32_t)((np + chunk - 1) / chunk);
}

namespace {
size_t al(size_t b) { return (b + 255) & ~(size_t)255; }
}  // namespace

uint32_t coa_msm_run(size_t n);

// Sized for the run length coa_msm_run(n) picks now (COA_MSM_RUN read at
// this call); coa_launch_msm refuses a workspace too small for its run.
size_t coa_msm_ws_bytes(size_t n) {
  const size_t np = 2 * n + 1;
  const size_t nc = coa_msm_chunks_run(n, coa_msm_run(n));
  return al(n * 32) + al(n * 16) + al(np * 128) + al((size_t)WA * dig_stride(np) * 2) + al(COA_MSM_PREP_BLOCKS * 36) +
         al((size_t)WA * nc * 128) + al((size_t)WA * 128) + al(16) + al((size_t)WA * nc * SEG_SLOTS * 128);
}

MsmWs coa_msm_ws_carve(void* base, size_t n) {
  const size_t np = 2 * n + 1;
  const size_t nc = coa_msm_chunks_run(n, coa_msm_run(n));
  char* p = static_cast<char*>(base);
  MsmWs w;
  w.nchunks_cap = (uint32_t)nc;
  w.k = reinterpret_cast<uint32_t*>(p);
  p += al(n * 32);
  w.z = reinterpret_cast<uint32_t*>(p);
  p += al(n * 16);
  w.pts = reinterpret_cast<uint32_t*>(p);
  p += al(np * 128);
  w.dig = reinterpret_cast<int16_t*>(p);
  p += al((size_t)WA * dig_stride(np) * 2);
  w.zpart = reinterpret_cast<uint32_t*>(p);
  p += al(COA_MSM_PREP_BLOCKS * 36);
  w.part = reinterpret_cast<uint32_t*>(p);
  p += al((size_t)WA * nc * 128);
  w.wsum = reinterpret_cast<uint32_t*>(p);
  p += al((size_t)WA * 128);
  w.bad = reinterpret_cast<uint32_t*>(p);
  p += al(16);
  w.segs = reinterpret_cast<uint32_t*>(p);
  return w;
}

// Sorted entries per lane: MAXRUN = 64 (16,384 points per workgroup, 36 KiB
// of LDS: three workgroups per CU at k_msm_bucket's 149 VGPRs) once that
// still gives >= 512 bucket workgroups, else fewer (down to 16) so small
// batches fill the 256 CUs.  For 2^21 signatures run 64 at three waves per
// SIMD took 4.07 ms against run 128 (32,768 points, 68 KiB, two workgroups
// per CU) at 4.28 ms.  (A run chosen in 64..128 to fill each XCD's last
// round -- 118, 6.0 rounds against 5.6 -- measured 4.42 ms against 4.38 at
// the two-wave build: the tails are not whole rounds.)  A group whose points fit one workgroup at
// run 16 takes the shortest run of at least 4 that still holds them: one
// certificate's 135 points, one group through these kernels, p50 0.388 ms at
// run 16, 0.353 at 8, 0.347 at 4, 0.374 at 2, 0.432 at 1 (tools/gpu_r3_k.sh:
// the lane runs are the serial part of a one-chunk window, but below 4 more
// entries become continuation segments the gather adds one by one).
// COA_MSM_RUN overrides (A/B runs).
// (chunk, window) pairs with points: the k_msm_bucket grid
static size_t bucket_pairs(size_t n, uint32_t run) {
  const size_t chunk = 256 * (size_t)run;
  const size_t nrc = n / chunk, nc = (2 * n + chunk) / chunk;
  return nrc * WR + (nc - nrc) * WA;
}

static uint32_t device_cus() {
  static std::atomic<uint32_t> cached{0};
  if (const uint32_t c = cached.load(std::memory_order_relaxed)) return c;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  cached.store((uint32_t)cus, std::memory_order_relaxed);
  return (uint32_t)cus;
}

uint32_t coa_msm_run(size_t n) {
  const char* e = getenv("COA_MSM_RUN");
  if (e) {
    const int r = atoi(e);
    if (r >= 1 && r <= MAXRUN) return (uint32_t)r;
  }
  if (2 * n + 1 <= 256 * 16) {
    uint32_t run = 4;
    while (256 * run < 2 * n + 1) run <<= 1;
    return run;
  }
  if (bucket_pairs(n, MAXRUN) >= 512) {
    // Large groups: the run in [3/4 MAXRUN, MAXRUN] with the fewest lane
    // steps, rounds x (run + 6), rounds = pairs over the workgroups resident
    // at once (three per CU): the workgroups now take equal time, so a last
    // round barely started costs nearly a whole one.  2^21 signatures: run
    // 59, 6,130 pairs in 7.98 rounds of 768, against run 64's 5,661 in 7.37
    // (k_msm_bucket 3.26 against 3.38 ms, the call 8.08 against 8.17 ms).
    const size_t slots = 3 * (size_t)device_cus();
    uint32_t best = MAXRUN;
    size_t best_cost = ~(size_t)0;
    for (uint32_t run = MAXRUN; run >= MAXRUN * 3 / 4; run--) {
      const size_t cost = (bucket_pairs(n, run) + slots - 1) / slots * (run + 6);
      if (cost < best_cost) {
        best_cost = cost;
        best = run;
      }
    }
    return best;
  }
  for (uint32_t run = MAXRUN / 2; run > 16; run >>= 1)
    if (bucket_pairs(n, run) >= 512) return run;
  return 16;
}

uint32_t coa_msm_chunks(size_t n) { return coa_msm_chunks_run(n, coa_msm_run(n)); }

// Dwords per point record (affine Niels, 24 dwords): padded to 32 by default
// so every record is one 128-byte line -- the bucket kernel reads them at
// random, and a 96-byte record straddles two lines three times in four.
// COA_MSM_PSTRIDE=24 packs them (A/B).
static uint32_t msm_pstride() {
  const char* e = getenv("COA_MSM_PSTRIDE");
  return (e && atoi(e) == 24) ? 24u : 32u;
}

hipError_t coa_launch_msm(const uint8_t* pks, const uint8_t* sigs, uint32_t n, const MsmWs& ws, uint8_t* verdict,
                          hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint32_t np = 2 * n + 1;
  const uint32_t run = coa_msm_run(n);
  const uint32_t nc = coa_msm_chunks_run(n, run);
  if (nc > ws.nchunks_cap) return hipErrorInvalidValue;  // COA_MSM_RUN changed since the workspace was sized
  hipError_t e = hipMemsetAsync(ws.bad, 0, 4, s);
  if (e != hipSuccess) return e;
  // small batches: a DPP row per point (the chain on 16 lanes, ~30 % less
  // latency); from 2,048 signatures one lane per point
  const bool rows = n <= 2048;
  uint32_t pb = (uint32_t)(((uint64_t)2 * n * (rows ? 16 : 1) + 255) / 256);
  if (pb > COA_MSM_PREP_BLOCKS) pb = COA_MSM_PREP_BLOCKS;
  const uint32_t ps = msm_pstride();
  // COA_MSM_TREE=0: sum_j j·B_j per (chunk, window) workgroup, then the chunk
  // partials per window (k_msm_wsum); default: the tree form (k_msm_bsum*)
  const char* te = getenv("COA_MSM_TREE");
  const uint32_t tree = (nc > 1 && !(te && atoi(te) == 0)) ? 1u : 0u;
  if (rows)
    hipLaunchKernelGGL(k_msm_prep<true>, dim3(pb), dim3(256), 0, s, pks, sigs, ws.k, ws.z, n, np, ws.pts, ws.dig,
                       ws.zpart, ws.bad, ps);
  else
    hipLaunchKernelGGL(k_msm_prep<false>, dim3(pb), dim3(256), 0, s, pks, sigs, ws.k, ws.z, n, np, ws.pts, ws.dig,
                       ws.zpart, ws.bad, ps);
  hipLaunchKernelGGL(k_msm_bpoint, dim3(1), dim3(256), 0, s, ws.zpart, pb, n, np, ws.pts, ws.dig, ps);
  // chunks holding R points only (z_i weights: WR windows)
  const uint32_t nrc = (uint32_t)(n / (256 * (size_t)run));
  const uint32_t g8 = (nrc * WR + (nc - nrc) * WA + 7) & ~7u;
  if (tree)
    hipLaunchKernelGGL(k_msm_bucket<true>, dim3(g8), dim3(256), 0, s, ws.pts, ws.dig, n, np, run, nc, nrc, ws.segs,
                       ws.part, ps);
  else
    hipLaunchKernelGGL(k_msm_bucket<false>, dim3(g8), dim3(256), 0, s, ws.pts, ws.dig, n, np, run, nc, nrc, ws.segs,
                       ws.part, ps);
  if (tree) {
    hipLaunchKernelGGL(k_msm_bsum1, dim3(WA * ((nc + kTreeGroup - 1) / kTreeGroup)), dim3(256), 0, s, ws.segs, nc,
                       nrc);
    hipLaunchKernelGGL(k_msm_bsum2, dim3(WA), dim3(256), 0, s, ws.segs, nc, ws.wsum);
  } else if (nc > 1) {
    // (one chunk, small groups: its partials already are the window sums,
    // laid out as wsum, window w at w * 32 words)
    hipLaunchKernelGGL(k_msm_wsum, dim3(WA), dim3(256), 0, s, ws.part, nc, nrc, ws.wsum);
  }
  hipLaunchKernelGGL(k_msm_final, dim3(1), dim3(64), 0, s, nc > 1 ? ws.wsum : ws.part, ws.bad, verdict);
  return hipGetLastError();
}
