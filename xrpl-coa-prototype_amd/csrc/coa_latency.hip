// Single-signature latency kernel for gfx950: crypto::Signature::verify ==
// ed25519-dalek 1.0.1 verify_strict (crypto/src/lib.rs:200-204), for callers
// that verify one message at a time -- Header::verify and Vote::verify
// (primary/src/messages.rs:64-66,139-141, from Core::process_header /
// process_vote, primary/src/core.rs:306-336).
//
// The throughput kernels (coa_halved.hip) give each signature ONE lane, so a
// lone signature waits for a whole one-lane verification (~0.9 ms).  Here one
// 256-thread workgroup (four waves, four SIMDs) works on one signature and
// the latency-bound chains run on 16-lane DPP rows (coa_fe_wave.h,
// coa_ge_rows.h):
//
//   key registered (coa_committee_register; committee keys are fixed per
//   config::Committee):
//     wave 0  k = SHA-512(R || A || M) mod l, then [k](-A) from the key's
//             radix-256 comb: one term per lane, summed by a 5-level butterfly
//     wave 2  [s]B from B's comb the same way (needs no hash, runs meanwhile)
//     wave 1  R's decompression, the power chain on the rows
//     meanwhile wave 0: P = [s]B + [k](-A), verify_strict's small-order test
//     of R taken on P (an accepting verdict needs R == P), and the half of
//     the compare that needs only P; wave 1 finishes decompression, compare
//     and verdict in two row products after its chain (coa_rcmp.h).
//   key not registered (the halved-scalar check of coa_halved.hip):
//     wave 0  k, the halving (c, d) with c == d k (mod 8l), e = d s mod l
//     wave 3  A's decompression (rows), small-order test, table j(-A), j <= 8
//     wave 1  the same for R
//     then, in parallel: wave 3 [c](-A) and wave 1 [|d|](-/+R) by signed
//     radix-16 Horner chains on the rows, wave 2 [e]B from B's comb; wave 0
//     sums the three and tests Q == O.
// Both verdicts are dalek's bit for bit: the cached one by the same argument
// as k_cert_verify_lat's header job, the uncached one by the halving argument
// of coa_halved.hip (Q == [d]P exactly, d odd).
// Batch prefilter (LatArgs::batch, Signature::verify_batch of small calls,
// crypto/src/lib.rs:206-219): the verdict also requires [l]A == O -- the
// registered key's flag, or for an unregistered key [l](-A) by wave 0 on
// wave 3's table while waves 1 and 3 run their chains.  Then an accepted vote
// satisfies R + (h mod l) A == [s]B and (z h mod l) A == z h A, so a group
// of accepted votes passes dalek's batch equation for every z; any other
// group is resolved by the exact batch kernels (coa_runtime.cpp).
// kernels here exceed the +-128 KiB reach of an out-of-line fold (coa_fe.h)
#define COA_RARE_INLINE
#include "coa_latency.h"

#include "coa_fe.h"
#include "coa_ge.h"
#include "coa_ge_rows.h"
#include "coa_halve.h"
#include "coa_halved.h"
#include "coa_committee.h"
#include "coa_keycache.h"
#include "coa_rcmp.h"
#include "coa_sc.h"
#include "coa_sha512.h"
#include "coa_smul.h"

namespace {
using namespace coa_kc;

// one comb term per lane (lanes 0..31; the upper half sums a copy) of the
// radix-256 comb `tab` for the 8-dword scalar dg, summed by an xor butterfly:
// every lane ends with sum_j tab[j][byte j of dg] (signed digits)
COA_DEV void comb_butterfly(ge_p3& P, uint32_t* dg, const uint32_t* tab, uint32_t lane) {
  add_const_word(dg, 0x80808080u);
  const int j = lane & 31;
  const int e = (int)byte_of(dg, j) - 128;
  ge_niels q;
  comb_select(q, tab, j, e);
  ge_p1p1 t;
  ge_p3_identity(P);
  ge_madd(t, P, q);
  ge_p1p1_to_p3(P, t);
#pragma unroll 1
  for (int off = 16; off >= 1; off >>= 1) {
    ge_p3 O;
    shfl_fe<64>(O.X, P.X, off);
    shfl_fe<64>(O.Y, P.Y, off);
    shfl_fe<64>(O.Z, P.Z, off);
    shfl_fe<64>(O.T, P.T, off);
    ge_cached oc;
    ge_p3_to_cached(oc, O);
    ge_add(t, P, oc);
    ge_p1p1_to_p3(P, t);
  }
}

COA_DEV void lds_put_p3(uint32_t* d, const ge_p3& P) {
  const fe* f[4] = {&P.X, &P.Y, &P.Z, &P.T};
#pragma unroll
  for (int q = 0; q < 4; q++)
#pragma unroll
    for (int i = 0; i < 8; i++) d[q * 8 + i] = f[q]->v[i];
}
COA_DEV void lds_get_p3(ge_p3& P, const uint32_t* d) {
  fe* f[4] = {&P.X, &P.Y, &P.Z, &P.T};
#pragma unroll
  for (int q = 0; q < 4; q++)
#pragma unroll
    for (int i = 0; i < 8; i++) f[q]->v[i] = d[q * 8 + i];
}

// row-form table entry: 4 coordinates x 8 limbs in LDS (row 0 writes)
COA_DEV void tab_put(uint32_t* e, const rp::Ca& c) {
  const uint32_t l = __lane_id();
  if (l < 8) {
    e[l] = c.ypx;
    e[8 + l] = c.ymx;
    e[16 + l] = c.Z;
    e[24 + l] = c.t2d;
  }
}
// entry |d| - 1 of the table (identity for d = 0), negated for d < 0
COA_DEV void tab_get(rp::Ca& c, const uint32_t* tab, int d) {
  const int m = d < 0 ? -d : d;
  const uint32_t l = __lane_id() & 15u;
  if (m == 0) {
    const uint32_t one = l == 0 ? 1u : 0u;
    c.ypx = one;
    c.ymx = one;
    c.Z = one;
    c.t2d = 0;
    return;
  }
  const uint32_t* e = tab + (m - 1) * 32;
  const uint32_t ypx = l < 8 ? e[l] : 0u, ymx = l < 8 ? e[8 + l] : 0u;
  c.Z = l < 8 ? e[16 + l] : 0u;
  const uint32_t t2d = l < 8 ? e[24 + l] : 0u;
  if (d < 0) {  // -(x, y) = (-x, y): swap Y+X and Y-X, negate 2dT
    c.ypx = ymx;
    c.ymx = ypx;
    c.t2d = fw::sub(0u, t2d);
  } else {
    c.ypx = ypx;
    c.ymx = ymx;
    c.t2d = t2d;
  }
}

// tab[j - 1] = j * (-Q), j = 1..8, in cached form (row arithmetic)
COA_DEV void build_table(uint32_t* tab, const ge_p3& Q) {
  rp::P1 base, cur;
  rp::L1 t;
  rp::from_p3(base, Q);
  rp::neg(cur, base);
  rp::Ca c1, cj;
  rp::to_cached(c1, cur);
  tab_put(tab, c1);
#pragma unroll 1
  for (int j = 1; j < 8; j++) {
    rp::add(t, cur, c1);
    rp::to_p3(cur, t);
    rp::to_cached(cj, cur);
    tab_put(tab + j * 32, cj);
  }
}

// sum_pos digit_pos 16^pos * table point, digits = nibble pos of rec minus 8
// (negated when neg), by a signed radix-16 Horner chain on the rows
COA_DEV void horner(ge_p3& out, const uint32_t* tab, const uint32_t* rec, int H, bool neg) {
  rp::P1 acc3;
  rp::L1 t;
  rp::P2 acc2;
  rp::identity(acc3);
  rp::Ca q;
#pragma unroll 1
  for (int pos = H - 1; pos >= 0; pos--) {
    int d = (int)((word_sel(rec, pos >> 3) >> (4 * (pos & 7))) & 15u) - 8;
    if (neg) d = -d;
    if (pos != H - 1) {
#pragma unroll 1
      for (int k = 0; k < 3; k++) {
        rp::dbl(t, acc2);
        rp::to_p2(acc2, t);
      }
      rp::dbl(t, acc2);
      rp::to_p3(acc3, t);
    }
    tab_get(q, tab, d);
    rp::add(t, acc3, q);
    if (pos != 0) rp::to_p2(acc2, t);
  }
  rp::to_p3(acc3, t);
  rp::to_ge_p3(out, acc3);
}

// The verdict straight into page-locked host memory, tagged with the call:
// the host polls for the tag instead of a device-to-host copy and a stream
// synchronisation (one PCIe write per signature).  The word is the whole
// message, so the store is relaxed: a release would first write back the L2
// (buffer_wbl2) for data nobody reads.
// A prefilter item of a certificate (LatArgs::cd_in): its message becomes
// Certificate::digest = SHA-512(id || round || origin)[..32] of the
// certificate whose index the record's first message dword holds.  Called by
// the wave that hashes k = H(R || A || M), before it does.
COA_DEV void cert_msg(const LatArgs& a, uint32_t item, uint32_t* msg) {
  if (!a.cd_in || item >= a.batch_n) return;
  const uint32_t* src = a.cd_in + (uint64_t)coa_sha::uni(msg[0]) * 18;
  uint32_t in[18];  // 72-byte records: 8-byte aligned only, so dword loads
#pragma unroll
  for (int i = 0; i < 18; i++) in[i] = coa_sha::uni(src[i]);
  uint64_t st[8];
  uint32_t h[16];
  coa_sha::hash_words<18>(st, in);
  coa_sha::state_to_le_words(h, st);
#pragma unroll
  for (int i = 0; i < 8; i++) msg[i] = h[i];
}

COA_DEV void publish(const LatArgs& a, uint32_t item, bool ok) {
  __hip_atomic_store(a.res + item, (a.tag << 8) | (ok ? 0u : 1u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// wave 0 of the uncached path: k = SHA-512(R || A || M) mod l, the halving
// (c, d), e = d s mod l (negated with d); the recoded c, d and e to sh_rec,
// the chain length, d's sign and s < l to sh_meta (lane 0); e stays in `e`
COA_DEV void halve_item(uint32_t* sh_rec, uint32_t* sh_meta, uint32_t* e_out, const uint32_t* msg,
                        const uint32_t* pk, const uint32_t* rw, const uint32_t* sw, uint32_t lane) {
  uint64_t st[8];
  uint32_t h[16], w[24];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    w[i] = rw[i];
    w[8 + i] = pk[i];
    w[16 + i] = msg[i];
  }
  coa_sha::hash_words<24>(st, w);
  coa_sha::state_to_le_words(h, st);
  sc k;
  sc_reduce512(k, h);
  uint32_t c[8], d[8];
  int cost;
  bool neg;
  coa_halve::halve(c, d, cost, neg, k.v);
  sc e;
  sc_mul(e, d, sw);  // s may be non-canonical here; the verdict rejects it
  if (neg) {
    sc en;
    sc_neg(en, e.v);
    e = en;
  }
  add_const_word(c, 0x88888888u);
  add_const_word(d, 0x88888888u);
#pragma unroll
  for (int i = 0; i < 8; i++) e_out[i] = e.v[i];
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      sh_rec[i] = c[i];
      sh_rec[8 + i] = d[i];
      sh_rec[16 + i] = e.v[i];
    }
    sh_meta[0] = (uint32_t)((cost + 2 + 3) / 4);  // c, |d| < 2^(4H - 2)
    sh_meta[1] = neg;
    sh_meta[2] = sc_is_canonical(sw);
  }
}

// waves 1 and 3: decompress the encoding on the rows and build the 8-entry
// table j(-Q); true when it decompresses and is not of small order
COA_DEV bool decompress_table(uint32_t* tab, const uint32_t* enc) {
  ge_p3 Q;
  const bool dec = ge_decompress<true>(Q, enc);
  const bool ok = dec && !ge_is_small_order(Q);
  build_table(tab, Q);
  return ok;
}

// Q + P0 + P1 == O (one-lane arithmetic; the points from LDS)
COA_DEV bool sum_is_identity(ge_p3 Q, const uint32_t* p0, const uint32_t* p1) {
  ge_p3 T;
  ge_cached c;
  ge_p1p1 t;
  const uint32_t* ps[2] = {p0, p1};
#pragma unroll 1
  for (int i = 0; i < 2; i++) {
    lds_get_p3(T, ps[i]);
    ge_p3_to_cached(c, T);
    ge_add(t, Q, c);
    ge_p1p1_to_p3(Q, t);
  }
  ge_p2 q2;
  ge_p3_to_p2(q2, Q);
  return ge_p2_is_identity(q2);
}

COA_DEV void flag_set(uint32_t* f) { __hip_atomic_store(f, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP); }
COA_DEV void flag_add(uint32_t* f) { __hip_atomic_fetch_add(f, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP); }
COA_DEV void flag_wait(uint32_t* f, uint32_t v) {
#pragma unroll 1
  while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < v) __builtin_amdgcn_s_sleep(1);
}

// The verify_batch prefilter on an unregistered key (LatArgs::batch): the
// halved-scalar verify_strict check of the barrier path, plus [l]A == O as
// [2^252]A == [l - 2^252](-A).  [2^252]A is a pure doubling chain (the
// kernel's longest: 252 doublings, two row products each) on wave 2 from
// its own decompression of A, started at once; wave 0 takes over wave 2's
// [e]B after the halving, then [l - 2^252](-A) (125 bits, 32 signed radix-16
// digits) on wave 3's table.  LDS flags instead of barriers, so no wave waits
// for a phase it does not need.  Same verdict as one 64-digit [l](-A) chain
// after the barrier, in ~0.8 of its time.
COA_DEV void uncached_batch(const LatArgs& a, uint32_t item, uint32_t wave, uint32_t lane, const uint32_t* msg,
                            const uint32_t* pk, const uint32_t* rw, const uint32_t* sw, uint32_t* sh_rec,
                            uint32_t* sh_ok, uint32_t (*sh_pt)[32], uint32_t (*sh_tab)[8 * 32]) {
  __shared__ uint32_t s_meta[4];
  __shared__ uint32_t s_flag[4];  // 0: sh_rec ready, 1: table j(-A) ready, 2: points published (count)
  __shared__ uint32_t s_big[32];  // [2^252]A
  if (threadIdx.x < 4) s_flag[threadIdx.x] = 0;
  __syncthreads();
  if (wave == 0) {
    uint32_t e[8], m[8];
#pragma unroll
    for (int i = 0; i < 8; i++) m[i] = msg[i];
    cert_msg(a, item, m);
    halve_item(sh_rec, s_meta, e, m, pk, rw, sw, lane);
    if (lane == 0) flag_set(&s_flag[0]);
    ge_p3 E;
    comb_butterfly(E, e, a.comb, lane);
    flag_wait(&s_flag[1], 1);
    uint32_t rec[8] = {0xe57e5c75u, 0xe09aeba2u, 0x2b80255eu, 0x9d678267u, 0, 0, 0, 0};  // (l - 2^252) + 0x88..8
    ge_p3 D;
    horner(D, sh_tab[0], rec, 32, false);  // D = [l - 2^252](-A)
    flag_wait(&s_flag[2], 3);
    bool ok = s_meta[2] != 0 && sh_ok[1] != 0 && sh_ok[3] != 0 && sum_is_identity(E, sh_pt[0], sh_pt[1]);
    // [l]A = [2^252]A - D
    ge_p3 big;
    lds_get_p3(big, s_big);
    fe_neg(D.X, D.X);
    fe_neg(D.T, D.T);
    ge_cached c;
    ge_p1p1 t;
    ge_p3_to_cached(c, D);
    ge_add(t, big, c);
    ge_p1p1_to_p3(big, t);
    ge_p2 b2;
    ge_p3_to_p2(b2, big);
    ok = ok && ge_p2_is_identity(b2);
    if (lane == 0) publish(a, item, ok);
  } else if (wave == 1 || wave == 3) {
    const bool ok = decompress_table(sh_tab[wave == 3 ? 0 : 1], wave == 3 ? pk : rw);
    if (lane == 0) {
      sh_ok[wave] = ok;
      if (wave == 3) flag_set(&s_flag[1]);
    }
    flag_wait(&s_flag[0], 1);
    const int H = (int)coa_sha::uni(s_meta[0]);
    const bool dneg = coa_sha::uni(s_meta[1]) != 0;
    uint32_t rec[8];
#pragma unroll
    for (int i = 0; i < 8; i++) rec[i] = coa_sha::uni(sh_rec[(wave == 3 ? 0 : 8) + i]);
    ge_p3 T;
    horner(T, sh_tab[wave == 3 ? 0 : 1], rec, H, wave == 1 && dneg);
    if (lane == 0) {
      lds_put_p3(sh_pt[wave == 3 ? 0 : 1], T);
      flag_add(&s_flag[2]);
    }
  } else {  // wave 2
    ge_p3 A;
    (void)ge_decompress<true>(A, pk);  // a failed decompression is wave 3's verdict
    rp::P1 acc3;
    rp::from_p3(acc3, A);
    rp::P2 acc2 = {acc3.X, acc3.Y, acc3.Z};
    rp::L1 t;
#pragma unroll 1
    for (int k = 0; k < 251; k++) {
      rp::dbl(t, acc2);
      rp::to_p2(acc2, t);
    }
    rp::dbl(t, acc2);
    rp::to_p3(acc3, t);
    ge_p3 big;
    rp::to_ge_p3(big, acc3);
    if (lane == 0) {
      lds_put_p3(s_big, big);
      flag_add(&s_flag[2]);
    }
  }
}

}  // namespace

#ifdef COA_VLAT_TRACE  // phase timestamps of item 0 per wave (tools/vlat_trace.py)
__device__ unsigned long long g_vlat_trace[4][8];
#define VMARK(i) \
  if (item == 0 && lane == 0) g_vlat_trace[wave][i] = clock64();
extern "C" int coa_vlat_trace(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_vlat_trace), sizeof(g_vlat_trace)) == hipSuccess ? 0 : -1;
}
#else
#define VMARK(i)
#endif

__global__ void __launch_bounds__(256) k_verify_lat(LatArgs a) {
  __shared__ uint32_t sh_rec[24];      // c' | d' | e (wave 0, uncached path)
  __shared__ uint32_t sh_meta[4];      // H, d < 0, s < l
  __shared__ uint32_t sh_ok[4];        // per wave: decompression ok and not small order
  __shared__ uint32_t sh_pt[3][32];    // points handed to wave 0
  __shared__ uint32_t sh_tab[2][8 * 32];  // j(-A), j(-R) in cached form (uncached path)
  const uint32_t wave = coa_sha::uni(threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t item = blockIdx.x;
  const uint32_t* in = item < a.n_inline ? a.inl[item] : a.in + (uint64_t)item * 32;
  uint32_t msg[8], pk[8], rw[8], sw[8];
  load8u(msg, in);
  load8u(pk, in + 8);
  load8u(rw, in + 16);
  load8u(sw, in + 24);
  VMARK(0)
  const int slot = a.nk ? key_lookup_u(a.keys, a.nk, pk) : -1;

  if (slot >= 0) {  // ------------------------------------------ cached key
    __shared__ uint32_t s_ready;  // wave 2 published [s]B
    __shared__ rcmp::Shared cmp;  // wave 0's half of the compare, for wave 1
    if (threadIdx.x == 0) {
      s_ready = 0;
      cmp.ready = 0;
    }
    __syncthreads();
    if (wave == 1) {  // R's decompression on the rows, the compare, the verdict
      uint32_t pre = 0;
      const uint32_t res = rcmp::decompress_eq(cmp, rw, pre);
      const bool tf = item >= a.batch_n || (coa_sha::uni(a.kflags[slot]) & COA_KEY_TORSION_FREE) != 0u;
      if (lane == 0) publish(a, item, pre == 0 && res == 3u && tf);
      VMARK(3)
    } else if (wave == 2) {  // [s]B on the rows, published in row-limb layout
      uint32_t dg[8];
#pragma unroll
      for (int i = 0; i < 8; i++) dg[i] = sw[i];
      rp::P1 S;
      rcmp::comb_sum_rows(S, dg, a.comb, lane);
      if (lane < 8) {
        sh_pt[0][lane] = S.X;
        sh_pt[0][8 + lane] = S.Y;
        sh_pt[0][16 + lane] = S.Z;
        sh_pt[0][24 + lane] = S.T;
      }
      if (lane == 0) __hip_atomic_store(&s_ready, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if (wave == 0) {
      uint64_t st[8];
      uint32_t h[16], w[24];
      cert_msg(a, item, msg);
#pragma unroll
      for (int i = 0; i < 8; i++) {
        w[i] = rw[i];
        w[8 + i] = pk[i];
        w[16 + i] = msg[i];
      }
      coa_sha::hash_words<24>(st, w);
      coa_sha::state_to_le_words(h, st);
      sc k;
      sc_reduce512(k, h);
      const uint32_t kf = coa_sha::uni(a.kflags[slot]);
      const uint32_t pre = (sc_is_canonical(sw) ? 0u : 1u) | ((kf & COA_KEY_DECOMPRESSES) ? 0u : 2u) |
                           ((kf & COA_KEY_SMALL_ORDER) ? 4u : 0u);
      rp::P1 P;
      rcmp::comb_sum_rows(P, k.v, a.ktabs + (uint64_t)slot * COA_KEY_TAB_DWORDS, lane);
      // everything that needs only P while wave 1 still decompresses R (the
      // critical chain): P = [s]B + [k](-A) once wave 2 has published [s]B,
      // verify_strict's small-order test of R taken on P (an accepting
      // verdict needs R == P, every other verdict is Err already), the
      // compare's P half
#pragma unroll 1
      while (__hip_atomic_load(&s_ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u)
        __builtin_amdgcn_s_sleep(1);
      rp::P1 S;
      S.X = rp::ld(sh_pt[0]);
      S.Y = rp::ld(sh_pt[0] + 8);
      S.Z = rp::ld(sh_pt[0] + 16);
      S.T = rp::ld(sh_pt[0] + 24);
      rcmp::add_rows(P, P, S);
      rcmp::prepare_rows(cmp, P, rw, pre, 8u, lane == 0);
    }
    VMARK(1)
    return;
  }

  // ------------------------------------------------------ uncached key
  if (item < a.batch_n) {  // verify_batch prefilter: the same check plus [l]A == O
    uncached_batch(a, item, wave, lane, msg, pk, rw, sw, sh_rec, sh_ok, sh_pt, sh_tab);
    return;
  }
  if (wave == 0) {
    uint32_t e[8];
    halve_item(sh_rec, sh_meta, e, msg, pk, rw, sw, lane);
  } else if (wave == 1 || wave == 3) {
    const bool ok = decompress_table(sh_tab[wave == 3 ? 0 : 1], wave == 3 ? pk : rw);
    if (lane == 0) sh_ok[wave] = ok;
  }
  VMARK(1)
  __syncthreads();
  VMARK(2)
  const int H = (int)coa_sha::uni(sh_meta[0]);
  const bool dneg = coa_sha::uni(sh_meta[1]) != 0;
  if (wave == 1 || wave == 3) {
    uint32_t rec[8];
#pragma unroll
    for (int i = 0; i < 8; i++) rec[i] = coa_sha::uni(sh_rec[(wave == 3 ? 0 : 8) + i]);
    ge_p3 T;
    horner(T, sh_tab[wave == 3 ? 0 : 1], rec, H, wave == 1 && dneg);
    if (lane == 0) lds_put_p3(sh_pt[wave == 3 ? 0 : 1], T);
  } else if (wave == 2) {
    uint32_t e[8];
#pragma unroll
    for (int i = 0; i < 8; i++) e[i] = coa_sha::uni(sh_rec[16 + i]);
    ge_p3 E;
    comb_butterfly(E, e, a.comb, lane);
    if (lane == 0) lds_put_p3(sh_pt[2], E);
  }
  VMARK(3)
  __syncthreads();
  VMARK(4)
  if (wave == 0) {
    ge_p3 Q;
    lds_get_p3(Q, sh_pt[2]);
    const bool ok = sh_meta[2] != 0 && sh_ok[1] != 0 && sh_ok[3] != 0 && sum_is_identity(Q, sh_pt[0], sh_pt[1]);
    if (lane == 0) publish(a, item, ok);
    VMARK(5)
  }
}

hipError_t coa_launch_verify_lat(const LatArgs& a, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_verify_lat, dim3(a.n), dim3(256), 0, s, a);
  return hipGetLastError();
}
