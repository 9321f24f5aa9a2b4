// Batch (random-linear-combination) verification for gfx950:
// crypto::Signature::verify_batch (crypto/src/lib.rs:206-219) ->
// ed25519-dalek 1.0.1 verify_batch.  One group = one certificate
// (Certificate::verify, primary/src/messages.rs:214).
//
// For a group with votes (A_i, R_i, s_i) over message M and weights z_i:
//   Ok  iff  every s_i < l, every A_i and R_i decompresses, and
//            [-(sum z_i s_i mod l)]B + sum [z_i]R_i + sum [z_i h_i mod l]A_i == O
//   with h_i = H(R_i || A_i || M) mod l.  No small-order rejection, no
//   cofactor -- exactly dalek.  The sum is computed exactly over the group,
//   so with the same z_i the verdict equals dalek's bit for bit, torsion
//   components included.
//
// Kernels:
//   k_batch_z       z_i = SHA-512("coa-batch-z" || seed || group || i || h_i || s_i)[0..16)
//   k_batch_terms   one lane per vote: validity flag and
//                   P_i = [z_i]R_i + [z_i h_i mod l]A_i + [-(z_i s_i) mod l]B
//                   by one joint Horner pass (signed radix-16 digits over two
//                   per-lane tables, signed radix-256 digits of the B scalar
//                   from the LDS B table); summing P_i over the group gives
//                   dalek's multiscalar sum term for term
//   k_batch_reduce  one workgroup per group: sum P_i (LDS tree), identity
//                   test, AND of the validity flags
#include "coa_batch.h"
#include "coa_kernels.h"

#include "coa_fe.h"
#include "coa_ge.h"
#include "coa_sc.h"
#include "coa_sha512.h"

#define BATCH_BLOCK 256

namespace {

// per-lane tables j·P (j = 1..8) for two bases, cached form, lane-major
// (2 KiB per lane; one 128-byte line per lookup, as in coa_kernels.hip):
//   uint4 index = ((lane * 16 + tab * 8 + entry) * 8 + quad)
COA_DEV void tab_store(uint32_t* scr, uint32_t lanes, uint32_t lane, int tab, int entry, const ge_cached& q) {
  const fe* f[4] = {&q.YplusX, &q.YminusX, &q.Z, &q.T2d};
#pragma unroll
  for (int c = 0; c < 4; c++)
#pragma unroll
    for (int h = 0; h < 2; h++) {
      uint4* dst = reinterpret_cast<uint4*>(scr) + (((uint64_t)lane * 16 + tab * 8 + entry) * 8 + c * 2 + h);
      *dst = make_uint4(f[c]->v[4 * h], f[c]->v[4 * h + 1], f[c]->v[4 * h + 2], f[c]->v[4 * h + 3]);
    }
}

COA_DEV void tab_select(ge_cached& q, const uint32_t* scr, uint32_t lanes, uint32_t lane, int tab, int d) {
  const int m = d < 0 ? -d : d;
  const int entry = m == 0 ? 0 : m - 1;
  fe* f[4] = {&q.YplusX, &q.YminusX, &q.Z, &q.T2d};
#pragma unroll
  for (int c = 0; c < 4; c++)
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint4 v =
          reinterpret_cast<const uint4*>(scr)[((uint64_t)lane * 16 + tab * 8 + entry) * 8 + c * 2 + h];
      f[c]->v[4 * h] = v.x;
      f[c]->v[4 * h + 1] = v.y;
      f[c]->v[4 * h + 2] = v.z;
      f[c]->v[4 * h + 3] = v.w;
    }
  if (m == 0) ge_cached_identity(q);
  ge_cached_cneg(q, d < 0);
}

COA_DEV void build_tab(uint32_t* scr, uint32_t lanes, uint32_t lane, int tab, const ge_p3& P) {
  ge_cached c1;
  ge_p3_to_cached(c1, P);
  tab_store(scr, lanes, lane, tab, 0, c1);
  ge_p3 cur = P;
#pragma unroll 1
  for (int j = 1; j < 8; j++) {
    ge_p1p1 t;
    ge_add(t, cur, c1);
    ge_p1p1_to_p3(cur, t);
    ge_cached cj;
    ge_p3_to_cached(cj, cur);
    tab_store(scr, lanes, lane, tab, j, cj);
  }
}

COA_DEV void add_const8(uint32_t* x, uint32_t c) {
  uint32_t cy = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) x[i] = addc32(x[i], c, cy, cy);
}
COA_DEV uint32_t top_byte(uint32_t* x) {
  const uint32_t top = x[7] >> 24;
#pragma unroll
  for (int i = 7; i > 0; i--) x[i] = (x[i] << 8) | (x[i - 1] >> 24);
  x[0] <<= 8;
  return top;
}

// Signed radix-256 digit e -> ±|e|·B from the LDS table (identity for 0).
COA_DEV void btab_niels(ge_niels& q, const uint32_t* lds, int e) {
  const int m = e < 0 ? -e : e;
  const int idx = m == 0 ? 0 : m - 1;
  const uint4* src = reinterpret_cast<const uint4*>(lds + idx * 24);
  uint32_t w[24];
#pragma unroll
  for (int i = 0; i < 6; i++) {
    const uint4 v = src[i];
    w[4 * i] = v.x;
    w[4 * i + 1] = v.y;
    w[4 * i + 2] = v.z;
    w[4 * i + 3] = v.w;
  }
#pragma unroll
  for (int i = 0; i < 8; i++) {
    q.yplusx.v[i] = w[i];
    q.yminusx.v[i] = w[8 + i];
    q.xy2d.v[i] = w[16 + i];
  }
  if (m == 0) ge_niels_identity(q);
  ge_niels_cneg(q, e < 0);
}

COA_DEV uint32_t top_nibble(uint32_t* x) {
  const uint32_t top = x[7] >> 28;
#pragma unroll
  for (int i = 7; i > 0; i--) x[i] = (x[i] << 4) | (x[i - 1] >> 28);
  x[0] <<= 4;
  return top;
}

}  // namespace

__global__ void __launch_bounds__(256) k_batch_z(const uint32_t* __restrict__ kbuf, const uint8_t* __restrict__ sigs,
                                                 const uint32_t* __restrict__ group_of, uint32_t group_const,
                                                 uint32_t n, uint64_t seed, uint32_t* __restrict__ zs) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    // one block: "coa-batch-z"(11) pad to 16 | seed 8 | group 4 | i 4 | h 32 | s 32 = 96 bytes
    uint32_t m[24];
    m[0] = 0x2d616f63u;  // "coa-"
    m[1] = 0x63746162u;  // "batc"
    m[2] = 0x007a2d68u;  // "h-z\0"
    m[3] = 0;
    m[4] = (uint32_t)seed;
    m[5] = (uint32_t)(seed >> 32);
    m[6] = group_of ? group_of[i] : group_const;
    m[7] = i;
#pragma unroll
    for (int j = 0; j < 8; j++) m[8 + j] = kbuf[(uint64_t)i * 8 + j];
    const uint32_t* sw = reinterpret_cast<const uint32_t*>(sigs + (uint64_t)i * 64 + 32);
#pragma unroll
    for (int j = 0; j < 8; j++) m[16 + j] = sw[j];
    uint64_t W[16];
#pragma unroll
    for (int w = 0; w < 12; w++) W[w] = coa_sha::be64(m[2 * w], m[2 * w + 1]);
    W[12] = 0x8000000000000000ull;
    W[13] = 0;
    W[14] = 0;
    W[15] = 96 * 8;
    uint64_t st[8];
    coa_sha::init(st);
    coa_sha::compress(st, W);
    uint32_t h[16];
    coa_sha::state_to_le_words(h, st);
#pragma unroll
    for (int j = 0; j < 4; j++) zs[(uint64_t)i * 4 + j] = h[j];
  }
}

// Per vote: flag (1 = valid encoding), P = [z]R + [z·h mod l]A + [-(z·s) mod l]B.
__global__ void __launch_bounds__(BATCH_BLOCK, 2) k_batch_terms(const uint8_t* __restrict__ pks,
                                                             const uint8_t* __restrict__ sigs,
                                                             const uint32_t* __restrict__ kbuf,
                                                             const uint32_t* __restrict__ zs, uint32_t n,
                                                             uint32_t* __restrict__ terms, uint8_t* __restrict__ flags,
                                                             uint32_t* __restrict__ scr,
                                                             const uint32_t* __restrict__ btab_g) {
  __shared__ __attribute__((aligned(16))) uint32_t btab[COA_BTAB_DWORDS];
  for (int t = threadIdx.x; t < COA_BTAB_DWORDS / 4; t += blockDim.x)
    reinterpret_cast<uint4*>(btab)[t] = reinterpret_cast<const uint4*>(btab_g)[t];
  __syncthreads();
  const uint32_t lanes = gridDim.x * blockDim.x;
  const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
  for (uint32_t i = lane; i < n; i += lanes) {
    uint32_t aw[8], rw[8], sw[8], hw[8], z[8];
    const uint32_t* pk = reinterpret_cast<const uint32_t*>(pks + (uint64_t)i * 32);
    const uint32_t* sg = reinterpret_cast<const uint32_t*>(sigs + (uint64_t)i * 64);
#pragma unroll
    for (int j = 0; j < 8; j++) {
      aw[j] = pk[j];
      rw[j] = sg[j];
      sw[j] = sg[8 + j];
      hw[j] = kbuf[(uint64_t)i * 8 + j];
      z[j] = j < 4 ? zs[(uint64_t)i * 4 + j] : 0;
    }
    bool ok = ((sw[7] & 0xe0000000u) == 0) && sc_is_canonical(sw);
    ge_p3 A, R;
#pragma unroll 1
    for (int which = 0; which < 2; which++) {
      uint32_t w[8];
#pragma unroll
      for (int j = 0; j < 8; j++) w[j] = which ? rw[j] : aw[j];
      ge_p3 P;
      ok = ge_decompress(P, w) && ok;
      if (which == 0) A = P;
      else R = P;
    }
    sc c, wz, nw;
    sc_mul(c, z, hw);   // z·h mod l
    sc_mul(wz, z, sw);  // z·s mod l
    sc_neg(nw, wz.v);   // -(z·s) mod l
    ge_p3 acc3;
    ge_p3_identity(acc3);
    if (ok) {
      build_tab(scr, lanes, lane, 0, R);
      build_tab(scr, lanes, lane, 1, A);
      uint32_t zp[8], cp[8], bp[8];
#pragma unroll
      for (int j = 0; j < 8; j++) {
        zp[j] = z[j];
        cp[j] = c.v[j];
        bp[j] = nw.v[j];
      }
      add_const8(zp, 0x88888888u);
      add_const8(cp, 0x88888888u);
      add_const8(bp, 0x80808080u);
      ge_p2 acc2;
      ge_p1p1 t;
#pragma unroll 1
      for (int d = 63; d >= 0; d--) {
        if (d != 63) {
#pragma unroll 1
          for (int dd = 0; dd < 3; dd++) {
            ge_p2_dbl(t, acc2);
            ge_p1p1_to_p2(acc2, t);
          }
          ge_p2_dbl(t, acc2);
          ge_p1p1_to_p3(acc3, t);
        }
        ge_cached q;
        tab_select(q, scr, lanes, lane, 0, (int)top_nibble(zp) - 8);
        ge_add(t, acc3, q);
        ge_p1p1_to_p3(acc3, t);
        tab_select(q, scr, lanes, lane, 1, (int)top_nibble(cp) - 8);
        ge_add(t, acc3, q);
        if ((d & 1) == 0) {
          const int e = (int)top_byte(bp) - 128;
          ge_niels qb;
          btab_niels(qb, btab, e);
          ge_p1p1_to_p3(acc3, t);
          ge_madd(t, acc3, qb);
        }
        if (d == 0) ge_p1p1_to_p3(acc3, t);
        else ge_p1p1_to_p2(acc2, t);
      }
    }
    // terms: X,Y,Z,T (32 dwords) per vote
    uint4* o = reinterpret_cast<uint4*>(terms + (uint64_t)i * 32);
    const fe* f[4] = {&acc3.X, &acc3.Y, &acc3.Z, &acc3.T};
#pragma unroll
    for (int q = 0; q < 4; q++) {
      o[2 * q] = make_uint4(f[q]->v[0], f[q]->v[1], f[q]->v[2], f[q]->v[3]);
      o[2 * q + 1] = make_uint4(f[q]->v[4], f[q]->v[5], f[q]->v[6], f[q]->v[7]);
    }
    flags[i] = ok ? 1 : 0;
  }
}

COA_DEV void load_p3(ge_p3& p, const uint32_t* src) {
#pragma unroll
  for (int j = 0; j < 8; j++) {
    p.X.v[j] = src[j];
    p.Y.v[j] = src[8 + j];
    p.Z.v[j] = src[16 + j];
    p.T.v[j] = src[24 + j];
  }
}
COA_DEV void store_p3(uint32_t* dst, const ge_p3& p) {
#pragma unroll
  for (int j = 0; j < 8; j++) {
    dst[j] = p.X.v[j];
    dst[8 + j] = p.Y.v[j];
    dst[16 + j] = p.Z.v[j];
    dst[24 + j] = p.T.v[j];
  }
}

// One workgroup per group: sum of the P_i, identity test, AND of the flags.
__global__ void __launch_bounds__(BATCH_BLOCK) k_batch_reduce(const uint64_t* __restrict__ offs,
                                                              const uint32_t* __restrict__ terms,
                                                              const uint8_t* __restrict__ flags,
                                                              uint8_t* __restrict__ verdicts) {
  __shared__ __attribute__((aligned(16))) uint32_t pts[BATCH_BLOCK * 32];
  __shared__ int bad;
  const uint32_t g = blockIdx.x;
  const uint64_t lo = offs[g], hi = offs[g + 1];
  const int tid = threadIdx.x;
  if (tid == 0) bad = 0;
  __syncthreads();
  ge_p3 acc;
  ge_p3_identity(acc);
  int mybad = 0;
  for (uint64_t i = lo + tid; i < hi; i += BATCH_BLOCK) {
    if (!flags[i]) mybad = 1;
    ge_p3 p;
    load_p3(p, terms + i * 32);
    ge_cached c;
    ge_p3_to_cached(c, p);
    ge_p1p1 t;
    ge_add(t, acc, c);
    ge_p1p1_to_p3(acc, t);
  }
  if (mybad) atomicOr(&bad, 1);
  store_p3(pts + tid * 32, acc);
  __syncthreads();
  for (int half = BATCH_BLOCK / 2; half > 0; half >>= 1) {
    if (tid < half) {
      ge_p3 a, b;
      load_p3(a, pts + tid * 32);
      load_p3(b, pts + (tid + half) * 32);
      ge_cached c;
      ge_p3_to_cached(c, b);
      ge_p1p1 t;
      ge_add(t, a, c);
      ge_p1p1_to_p3(a, t);
      store_p3(pts + tid * 32, a);
    }
    __syncthreads();
  }
  if (tid == 0) {
    ge_p2 r;
    r.X.v[0] = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      r.X.v[j] = pts[j];
      r.Y.v[j] = pts[8 + j];
      r.Z.v[j] = pts[16 + j];
    }
    verdicts[g] = (ge_p2_is_identity(r) && !bad) ? 0 : 1;
  }
}

hipError_t coa_launch_batch_z(const uint32_t* kbuf, const uint8_t* sigs, const uint32_t* group_of,
                              uint32_t group_const, uint32_t n, uint64_t seed, uint32_t* zs, hipStream_t s) {
  if (n == 0) return hipSuccess;
  uint32_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(k_batch_z, dim3(blocks), dim3(256), 0, s, kbuf, sigs, group_of, group_const, n, seed, zs);
  return hipGetLastError();
}

hipError_t coa_launch_batch_terms(const uint8_t* pks, const uint8_t* sigs, const uint32_t* kbuf, const uint32_t* zs,
                                  uint32_t n, uint32_t* terms, uint8_t* flags, uint32_t* scratch,
                                  uint32_t scratch_lanes, const uint32_t* btab, hipStream_t s) {
  if (n == 0) return hipSuccess;
  uint64_t blocks = (n + BATCH_BLOCK - 1) / BATCH_BLOCK;
  const uint64_t maxb = scratch_lanes / BATCH_BLOCK;
  if (blocks > maxb) blocks = maxb;
  hipLaunchKernelGGL(k_batch_terms, dim3((uint32_t)blocks), dim3(BATCH_BLOCK), 0, s, pks, sigs, kbuf, zs, n, terms,
                     flags, scratch, btab);
  return hipGetLastError();
}

hipError_t coa_launch_batch_reduce(const uint64_t* offs, uint32_t n_groups, const uint32_t* terms,
                                   const uint8_t* flags, uint8_t* verdicts, hipStream_t s) {
  if (n_groups == 0) return hipSuccess;
  hipLaunchKernelGGL(k_batch_reduce, dim3(n_groups), dim3(BATCH_BLOCK), 0, s, offs, terms, flags, verdicts);
  return hipGetLastError();
}
