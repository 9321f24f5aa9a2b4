// Committee key cache and the fused Certificate::verify
// kernel (f3) for gfx950.
//
// The reference re-decompresses every voter key on every call
// (crypto/src/lib.rs:202,216) although keys are fixed per Committee
// (config/src/lib.rs:140-143).  coa_committee_register() precomputes, once
// per committee and per device:
//   k_key_flags    decompression verdict, small order ([8]A == O) and
//                  torsion freedom ([l]A == O) of every key
//   k_key_tables   a comb of -A per key: entry (j, v) = (v+1)*256^j*(-A) as
//                  affine Niels, built by exact double-and-add, so torsion
//                  components are kept (the comb is an integer multiple, never
//                  reduced mod l)
// With those, a signature's equation P = [s]B + [k](-A) needs no doubling:
// 32 comb additions for each scalar (signed radix-256 digits).
//
// k_cert_verify runs the whole crypto of Certificate::verify
// (primary/src/messages.rs:189-215) in one launch, every check independent:
//   * header digest role (leading blocks, one lane per certificate):
//     SHA-512(Header::digest bytes)[..32] == header.id   (messages.rs:49-51)
//   * signature role, one job per header signature and per vote:
//     header: verify_strict(header.id, author)            (messages.rs:64-66)
//             -- s < l, A and R decompress, neither small order, P == R
//     vote:   the message is Certificate::digest =
//             SHA-512(id || round || origin)[..32]         (messages.rs:226-234)
//             computed in-kernel; per vote s < l, A and R decompress and
//             P == R (cofactorless, projective).
// verify_batch exactness (crypto/src/lib.rs:206-219 -> dalek verify_batch):
// dalek accepts iff sum z_i (R_i + h_i A_i - s_i B) == O for its random z_i,
// when every A_i is torsion free (then (z_i h_i mod l) A_i == z_i h_i A_i).
// So if every vote satisfies its own equation and every key is torsion free
// the batch verdict is Ok for EVERY z -- exactly dalek's.  Any other outcome
// with well-formed inputs is flagged COA_CST_VOTES_INCONCLUSIVE and the host
// re-runs that certificate through the exact RLC kernels (coa_batch.hip) with
// real weights; malformed inputs (s >= l, R or A not decompressing) are a
// definitive Err, as in dalek.
//
// Two variants:
//   k_cert_verify      throughput: two waves per SIMD, each lane a strided
//                      set of signatures (64 serial mixed additions each), P
//                      compared with R's encoding after one inversion shared
//                      by the lane's signatures; one lane per header digest
//   k_cert_verify_lat  latency: one 192-thread workgroup per signature --
//                      wave 0 hashes Certificate::digest and k, takes one
//                      term of [k](-A)'s comb per lane (32 lanes) and sums
//                      them by a 5-level xor butterfly; wave 2 does the same
//                      for [s]B meanwhile (it needs no hash); wave 1
//                      decompresses R on DPP rows (coa_fe_wave.h).  The
//                      three meet in LDS: P = both halves, small-order test,
//                      compare with R.  One
//                      workgroup per header digest: its lanes expand every
//                      block's message schedule into LDS, then one wave
//                      runs the rounds (coa_sha512.h, compress_kw).
// kernels here exceed the +-128 KiB reach of an out-of-line fold (coa_fe.h)
#define COA_RARE_INLINE
#include "coa_committee.h"

#include <cstddef>
#include <cstdlib>

#include "coa_fe.h"
#include "coa_ge.h"
#include "coa_halved.h"
#include "coa_sc.h"
#include "coa_keycache.h"
#include "coa_rcmp.h"
#include "coa_sha512.h"
#include "coa_smul.h"

namespace {
using namespace coa_kc;

COA_DEV void ge_neg(ge_p3& r, const ge_p3& p) {
  r = p;
  fe_neg(r.X, p.X);
  fe_neg(r.T, p.T);
}

// [m]P by MSB-first double-and-add over bits top..0 of m: an exact integer
// multiple (registration only; latency is irrelevant there).
COA_DEV void ge_mul_bits(ge_p3& out, const ge_p3& P, const uint32_t* m, int top) {
  ge_cached Pc;
  ge_p3_to_cached(Pc, P);
  ge_p3 acc;
  ge_p3_identity(acc);
  ge_p1p1 t;
#pragma unroll 1
  for (int b = top; b >= 0; b--) {
    ge_p3_dbl(t, acc);
    ge_p1p1_to_p3(acc, t);
    if ((word_sel(m, b >> 5) >> (b & 31)) & 1u) {
      ge_add(t, acc, Pc);
      ge_p1p1_to_p3(acc, t);
    }
  }
  out = acc;
}

COA_DEV void store_niels(uint32_t* e, const ge_p3& P) {
  fe zi, x, y, xy, d2, n0, n1, n2;
  fe_invert(zi, P.Z);
  fe_mul(x, P.X, zi);
  fe_mul(y, P.Y, zi);
  fe_mul(xy, x, y);
  fe_const_d2(d2);
  fe_add(n0, y, x);
  fe_sub(n1, y, x);
  fe_mul(n2, xy, d2);
  fe_canon(n0, n0);
  fe_canon(n1, n1);
  fe_canon(n2, n2);
  uint4* o = reinterpret_cast<uint4*>(e);
  o[0] = make_uint4(n0.v[0], n0.v[1], n0.v[2], n0.v[3]);
  o[1] = make_uint4(n0.v[4], n0.v[5], n0.v[6], n0.v[7]);
  o[2] = make_uint4(n1.v[0], n1.v[1], n1.v[2], n1.v[3]);
  o[3] = make_uint4(n1.v[4], n1.v[5], n1.v[6], n1.v[7]);
  o[4] = make_uint4(n2.v[0], n2.v[1], n2.v[2], n2.v[3]);
  o[5] = make_uint4(n2.v[4], n2.v[5], n2.v[6], n2.v[7]);
}

// certificate owning vote vi: the last c with voff[c] <= vi
COA_DEV uint32_t vote_cert(const uint64_t* __restrict__ voff, uint32_t nc, uint32_t vi) {
  uint32_t lo = 0, hi = nc;  // voff[lo] <= vi < voff[hi]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (voff[mid] <= vi) lo = mid;
    else hi = mid;
  }
  return lo;
}

COA_DEV uint32_t vote_cert_u(const uint64_t* __restrict__ voff, uint32_t nc, uint32_t vi) {
  uint32_t lo = 0, hi = nc;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (uni64(voff[mid]) <= vi) lo = mid;
    else hi = mid;
  }
  return lo;
}

// Throughput path, phase A of one signature job: flags and
// P = [s]B + [k](-A) from the combs (no doubling).  pre: bit0 s >= l, bit1 A
// does not decompress, bit2 A small order, bit3 A has torsion, bit4 header
// signature, bit5 key not registered, bit6 no job.
#define PRE_S 1u
#define PRE_A 2u
#define PRE_SMALL_A 4u
#define PRE_TORSION 8u
#define PRE_HDR 16u
#define PRE_UNCACHED 32u
#define PRE_NONE 64u

// p or q as a plain integer select (a ternary over two kernel-argument
// pointers is lowered through a private two-entry array, i.e. scratch)
COA_DEV const uint32_t* sel_ptr(bool c, const uint32_t* p, const uint32_t* q) {
  return reinterpret_cast<const uint32_t*>(c ? reinterpret_cast<uintptr_t>(p) : reinterpret_cast<uintptr_t>(q));
}

COA_DEV void job_comb(const CertArgs& a, uint32_t job, ge_p3& P, uint32_t& pre, uint32_t& cert) {
  const bool hdr = job < a.nc;
  const uint32_t vi = job - a.nc;
  const uint32_t c = hdr ? job : vote_cert(a.voff, a.nc, vi);
  cert = c;
  const uint32_t* sig = sel_ptr(hdr, a.hsigs + (uint64_t)c * 16, a.vsigs + (uint64_t)vi * 16);
  uint32_t pk[8], rw[8], sw[8], msg[8];
  load8(pk, sel_ptr(hdr, a.origins + (uint64_t)c * 8, a.vpks + (uint64_t)vi * 8));
  load8(rw, sig);
  load8(sw, sig + 8);
  load8(msg, a.ids + (uint64_t)c * 8);
  ge_p3_identity(P);
  const int slot = key_lookup(a.keys, a.nk, pk);
  if (slot < 0) {
    pre = PRE_UNCACHED;
    return;
  }
  uint64_t st[8];
  uint32_t h[16];
  if (!hdr && a.cdig) {  // Certificate::digest from the prologue kernel
    load8(msg, a.cdig + (uint64_t)c * 8);
  } else if (!hdr) {  // Certificate::digest = SHA-512(id || round u64 LE || origin)[..32]
    uint32_t in[18];
    const uint64_t rd = a.rounds[c];
#pragma unroll
    for (int i = 0; i < 8; i++) in[i] = msg[i];
    in[8] = (uint32_t)rd;
    in[9] = (uint32_t)(rd >> 32);
    load8(in + 10, a.origins + (uint64_t)c * 8);
    coa_sha::hash_words<18>(st, in);
    coa_sha::state_to_le_words(h, st);
#pragma unroll
    for (int i = 0; i < 8; i++) msg[i] = h[i];
  }
  {  // k = SHA-512(R || A || M) mod l
    uint32_t in[24];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      in[i] = rw[i];
      in[8 + i] = pk[i];
      in[16 + i] = msg[i];
    }
    coa_sha::hash_words<24>(st, in);
    coa_sha::state_to_le_words(h, st);
  }
  sc k;
  sc_reduce512(k, h);
  const uint32_t kf = a.kflags[slot];
  pre = (sc_is_canonical(sw) ? 0u : PRE_S) | ((kf & COA_KEY_DECOMPRESSES) ? 0u : PRE_A) |
        ((kf & COA_KEY_SMALL_ORDER) ? PRE_SMALL_A : 0u) | ((kf & COA_KEY_TORSION_FREE) ? 0u : PRE_TORSION) |
        (hdr ? PRE_HDR : 0u);
  // terms t < 32: B-comb bytes of s; t >= 32: key-comb bytes of k (signed
  // radix-256 digits = bytes of x + 0x80..80)
  uint32_t sd[8], kd[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    sd[i] = sw[i];
    kd[i] = k.v[i];
  }
  add_const_word(sd, 0x80808080u);
  add_const_word(kd, 0x80808080u);
  const uint32_t* ktab = a.ktabs + (uint64_t)slot * COA_KEY_TAB_DWORDS;
  ge_p1p1 t;
  // [s]B: 13 additions from the wide HBM comb when it is built, else the 32
  // byte terms of the radix-256 comb (an s >= l only reaches Err verdicts);
  // [k](-A): 13 or 16 additions from the key's wide comb (radix 2^20 or
  // 2^16) when the committee has them, else its 32 radix-256 terms
  if (a.wcomb) {
    wcomb_accumulate(P, sw, a.wcomb);
  } else {
#pragma unroll 1
    for (int j = 0; j < 32; j++) {
      ge_niels q;
      comb_select(q, a.comb, j, (int)byte_of(sd, j) - 128);
      ge_madd(t, P, q);
      ge_p1p1_to_p3(P, t);
    }
  }
  if (a.kwtabs && a.kw20) {
    wc_accumulate<COA_KWCOMB20_W, COA_KWCOMB20_POS, COA_KWC_STRIDE>(P, k.v, a.kwtabs + (uint64_t)slot * COA_KWCOMB20_DWORDS);
  } else if (a.kwtabs) {
    wc_accumulate<COA_KWCOMB_W, COA_KWCOMB_POS, COA_KWC_STRIDE>(P, k.v, a.kwtabs + (uint64_t)slot * COA_KWCOMB_DWORDS);
  } else {
#pragma unroll 1
    for (int j = 0; j < 32; j++) {
      ge_niels q;
      comb_select(q, ktab, j, (int)byte_of(kd, j) - 128);
      ge_madd(t, P, q);
      ge_p1p1_to_p3(P, t);
    }
  }
}

// Phase C: the verdict bits of a job from P's affine coordinates.  dalek's
// `P == decompress(R)` holds iff y_P == y_R (mod p; R's y is read as 255 bits,
// y >= p meaning y - p) and, unless x_P == 0, x_P's sign equals R's sign bit:
// when y_P == y_R the point P itself proves that R decompresses (to +-x_P).
COA_DEV uint32_t job_verdict(const CertArgs& a, uint32_t job, uint32_t pre, const fe& x, const fe& y) {
  if (pre & (PRE_NONE | PRE_UNCACHED)) return (pre & PRE_UNCACHED) ? COA_CST_UNCACHED : 0u;
  const bool hdr = (pre & PRE_HDR) != 0;
  const uint32_t* sig = sel_ptr(hdr, a.hsigs + (uint64_t)job * 16, a.vsigs + (uint64_t)(job - a.nc) * 16);
  uint32_t rw[8];
  load8(rw, sig);
  fe yr, xc, yc;
  fe_from_words(yr, rw);
  fe_canon(yr, yr);
  fe_canon(xc, x);
  fe_canon(yc, y);
  bool same_y = true, x_zero = true;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    same_y = same_y && yc.v[i] == yr.v[i];
    x_zero = x_zero && xc.v[i] == 0;
  }
  const bool eq = same_y && (x_zero || (xc.v[0] & 1u) == (rw[7] >> 31));
  const bool s_ok = !(pre & PRE_S), a_ok = !(pre & PRE_A);
  if (hdr) {
    // verify_strict: R == P, neither A nor R (== P) small order
    fe xx, yy, ss;
    fe_sq(xx, xc);
    fe_sq(yy, yc);
    fe_add(ss, xx, yy);
    bool y_zero = true;
#pragma unroll
    for (int i = 0; i < 8; i++) y_zero = y_zero && yc.v[i] == 0;
    const bool small_p = x_zero || y_zero || fe_iszero(ss);
    return (s_ok && a_ok && !(pre & PRE_SMALL_A) && eq && !small_p) ? 0u : COA_CST_BAD_HEADER_SIG;
  }
  if (!(s_ok && a_ok)) return COA_CST_BAD_VOTES;
  // P != R: R may not decompress (Err) or differ by a torsion point (a
  // weight-dependent verdict) -- the host's exact RLC path decides both
  return (eq && !(pre & PRE_TORSION)) ? 0u : COA_CST_VOTES_INCONCLUSIVE;
}

// Scratch slab of the throughput kernel: per job slot 9 uint4 rows, each row
// lane-major (row r of slot q at uint4 index (q * 9 + r) * lanes + lane):
// X, Y, Z, prefix product of the Z's (2 rows each), then (pre, cert, -, -).
#define PSCR_ROWS 9
COA_DEV void pscr_put(uint32_t* pscr, uint64_t lanes, uint64_t lane, int j, int row, const fe& f) {
#pragma unroll
  for (int h = 0; h < 2; h++)
    reinterpret_cast<uint4*>(pscr)[((uint64_t)j * PSCR_ROWS + row + h) * lanes + lane] =
        make_uint4(f.v[4 * h], f.v[4 * h + 1], f.v[4 * h + 2], f.v[4 * h + 3]);
}
COA_DEV void pscr_get(fe& f, const uint32_t* pscr, uint64_t lanes, uint64_t lane, int j, int row) {
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const uint4 v = reinterpret_cast<const uint4*>(pscr)[((uint64_t)j * PSCR_ROWS + row + h) * lanes + lane];
    f.v[4 * h] = v.x;
    f.v[4 * h + 1] = v.y;
    f.v[4 * h + 2] = v.z;
    f.v[4 * h + 3] = v.w;
  }
}

}  // namespace

// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_key_flags(const uint32_t* __restrict__ keys, uint32_t nk,
                                                   uint32_t* __restrict__ flags) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nk) return;
  uint32_t w[8];
  load8(w, keys + (uint64_t)i * 8);
  ge_p3 A;
  uint32_t f = 0;
  if (ge_decompress(A, w)) {
    f |= COA_KEY_DECOMPRESSES;
    if (ge_is_small_order(A)) f |= COA_KEY_SMALL_ORDER;
    uint32_t l[8];
    sc_const_l(l);
    ge_p3 LA;
    ge_mul_bits(LA, A, l, 252);
    ge_p2 q;
    ge_p3_to_p2(q, LA);
    if (ge_p2_is_identity(q)) f |= COA_KEY_TORSION_FREE;
  }
  flags[i] = f;
}

// one lane per table entry: (key, j, v) -> (v+1)*256^j*(-A)
__global__ void __launch_bounds__(256) k_key_tables(const uint32_t* __restrict__ keys, uint32_t nk,
                                                    uint32_t* __restrict__ tabs) {
  const uint64_t id = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t key = (uint32_t)(id / COA_KEY_TAB_ENTRIES);
  if (key >= nk) return;
  const uint32_t e = (uint32_t)(id % COA_KEY_TAB_ENTRIES), j = e >> 7, v = e & 127;
  uint32_t w[8];
  load8(w, keys + (uint64_t)key * 8);
  uint32_t* out = tabs + (uint64_t)key * COA_KEY_TAB_DWORDS + (uint64_t)e * 24;
  ge_p3 A;
  if (!ge_decompress(A, w)) {  // never selected by an accepting path; keep it a valid point
    ge_p3_identity(A);
  }
  ge_p3 nA, M;
  ge_neg(nA, A);
  uint32_t m[8];
#pragma unroll
  for (int i = 0; i < 8; i++) m[i] = 0;
  // (v+1) << 8j with v+1 <= 128: at most two dwords are nonzero
  const uint64_t sh = (uint64_t)(v + 1) << ((8 * j) & 31);
#pragma unroll
  for (int i = 0; i < 8; i++) {
    if (i == (int)((8 * j) >> 5)) m[i] = (uint32_t)sh;
    if (i == (int)((8 * j) >> 5) + 1) m[i] = (uint32_t)(sh >> 32);
  }
  ge_mul_bits(M, nA, m, 8 * j + 7);
  store_niels(out, M);
}

// Prologue of the throughput variant: Certificate::digest = SHA-512(id ||
// round u64 LE || origin)[..32] once per certificate (primary/src/
// messages.rs:226-234), instead of once per vote in the signature jobs (a
// C3 certificate has 67 votes: one SHA-512 block each saved).
__global__ void __launch_bounds__(256) k_cert_digests(CertArgs a, uint32_t* __restrict__ out) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= a.nc) return;
  uint32_t in[18];
  load8(in, a.ids + (uint64_t)c * 8);
  const uint64_t rd = a.rounds[c];
  in[8] = (uint32_t)rd;
  in[9] = (uint32_t)(rd >> 32);
  load8(in + 10, a.origins + (uint64_t)c * 8);
  uint64_t st[8];
  coa_sha::hash_words<18>(st, in);
  uint32_t h[16];
  coa_sha::state_to_le_words(h, st);
  uint4* o = reinterpret_cast<uint4*>(out + (uint64_t)c * 8);
  o[0] = make_uint4(h[0], h[1], h[2], h[3]);
  o[1] = make_uint4(h[4], h[5], h[6], h[7]);
}

// Throughput variant.  The leading blocks hash the header digests, one lane
// per certificate (SHA-512 of the Header::digest bytes, ~27 blocks at C3),
// beside the signature waves.  The signature waves are a persistent grid of
// two waves per SIMD that take chunks of 64 consecutive jobs (one per lane)
// from a global counter until none is left, so every SIMD stays busy to
// within one chunk of the end: a static split leaves some SIMDs with one
// chunk more than others (5 vs 6 at C3, ~15 %), and the signature waves the
// header waves displace start late and simply take fewer chunks.
// Phase A computes each job's P and parks it with the running product of the
// Z's in a lane-major scratch slab; ONE field inversion serves all of a
// lane's jobs (Montgomery's trick), then phase C compares each affine P with
// its R encoding.  Per vote: ~265/jobs field operations of inversion instead
// of R's ~277-operation decompression.  pscr[0] is the chunk counter (zeroed
// by the launcher); the slab holds jcap jobs per lane.
template <int WAVES>
__global__ void __launch_bounds__(256, WAVES) k_cert_verify(CertArgs a, uint32_t* __restrict__ pscr, uint32_t jcap) {
  if (blockIdx.x < a.hdr_blocks) {  // header digest role, one lane per certificate
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= a.nc) return;
    const uint64_t o0 = a.hdr_off[c], o1 = a.hdr_off[c + 1];
    uint64_t st[8];
    coa_sha::hash_mem(st, a.hdr_data + o0, o1 - o0);
    uint32_t h[16], id[8];
    coa_sha::state_to_le_words(h, st);
    load8(id, a.ids + (uint64_t)c * 8);
    bool same = true;
#pragma unroll
    for (int i = 0; i < 8; i++) same = same && h[i] == id[i];
    if (!same) atomicOr(a.status + c, COA_CST_BAD_HEADER_ID);
    return;
  }
  const uint64_t lanes = (uint64_t)(gridDim.x - a.hdr_blocks) * blockDim.x;
  const uint64_t lane = (uint64_t)(blockIdx.x - a.hdr_blocks) * blockDim.x + threadIdx.x;
  const uint32_t sub = threadIdx.x & 63;
  uint32_t* ctr = pscr;
  uint32_t* slab = pscr + 64;
  const uint64_t jobs = (uint64_t)a.nc + a.nv;
  const uint32_t chunks = (uint32_t)((jobs + 63) / 64);
  int nj = 0;  // this wave's chunks (the same for all its lanes)
  fe zp;       // running prefix product of the Z's
#pragma unroll 1
  for (;;) {
    if (nj >= (int)jcap) break;  // slab full: the other waves take the rest
    uint32_t chunk = 0;
    if (sub == 0) chunk = atomicAdd(ctr, 1u);
    chunk = __builtin_amdgcn_readfirstlane(__shfl(chunk, 0));
    if (chunk >= chunks) break;
    uint64_t job = (uint64_t)chunk * 64 + sub;
    if (a.perm && job < jobs) job = a.perm[job];  // key order (k_job_count, k_job_place)
    ge_p3 P;
    uint32_t pre = PRE_NONE, cert = 0;
    if (job < jobs) job_comb(a, (uint32_t)job, P, pre, cert);
    else ge_p3_identity(P);
    if (nj == 0) zp = P.Z;
    else fe_mul(zp, zp, P.Z);
    pscr_put(slab, lanes, lane, nj, 0, P.X);
    pscr_put(slab, lanes, lane, nj, 2, P.Y);
    pscr_put(slab, lanes, lane, nj, 4, P.Z);
    pscr_put(slab, lanes, lane, nj, 6, zp);
    reinterpret_cast<uint4*>(slab)[((uint64_t)nj * PSCR_ROWS + 8) * lanes + lane] =
        make_uint4(pre, cert, (uint32_t)job, 0);
    nj++;
  }
  if (nj == 0) return;
  fe inv;
  fe_invert(inv, zp);
#pragma unroll 1
  for (int j = nj - 1; j >= 0; j--) {
    fe zinv, x, y, X, Y;
    if (j > 0) {
      fe Z, zprev;
      pscr_get(zprev, slab, lanes, lane, j - 1, 6);
      pscr_get(Z, slab, lanes, lane, j, 4);
      fe_mul(zinv, inv, zprev);
      fe_mul(inv, inv, Z);
    } else {
      zinv = inv;
    }
    pscr_get(X, slab, lanes, lane, j, 0);
    pscr_get(Y, slab, lanes, lane, j, 2);
    const uint4 m = reinterpret_cast<const uint4*>(slab)[((uint64_t)j * PSCR_ROWS + 8) * lanes + lane];
    fe_mul(x, X, zinv);
    fe_mul(y, Y, zinv);
    const uint32_t bits = job_verdict(a, m.z, m.x, x, y);
    if (bits) atomicOr(a.status + m.y, bits);
  }
}

// ---------------------------------------------------------------------------
// Latency variant (one certificate at a time): see the file comment.
// Blocks [0, nc): header digests (wave 0 of each).  Blocks [nc, 2nc + nv):
// one signature job each.
#define KW_CHUNK 64  // blocks of schedule per LDS pass (40 KiB)
#ifdef COA_LAT_TRACE  // phase timestamps of the first signature job (tools/lat_trace.py)
__device__ unsigned long long g_lat_trace[3][8];
#define LAT_MARK(w, i) \
  if (job == 0 && lane == 0) g_lat_trace[w][i] = clock64();
extern "C" int coa_lat_trace(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lat_trace), sizeof(g_lat_trace)) == hipSuccess ? 0 : -1;
}
// header-digest block of certificate 0 and the kernel's end, in the
// GPU-wide 100 MHz real-time clock (comparable across CUs): 0 start, 1
// schedule expanded, 2 rounds done, 3 compared, 5 signature job 0's verdict,
// 6 the last block's publish, 7 signature job 0's start
__device__ unsigned long long g_hdr_trace[12];
#define HDR_MARK(i) g_hdr_trace[i] = __builtin_amdgcn_s_memrealtime();
extern "C" int coa_lat_trace_hdr(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_hdr_trace), sizeof(g_hdr_trace)) == hipSuccess ? 0 : -1;
}
#else
#define LAT_MARK(w, i)
#define HDR_MARK(i)
#endif
// One block's end of the latency kernel (one thread): OR its status bits
// into certificate c's word and, with a.host_res set, count itself done; the
// block that finishes last publishes every certificate's status word into
// page-locked host memory, tagged with the call (the host polls for the tag:
// no device-to-host copy, no stream synchronisation), and resets the status
// words and the block counter for the next call.
// Every value that crosses blocks is an atomic on its own word, so no fence
// orders other memory: the OR is a returning atomic whose completion the
// block waits for (s_waitcnt) before its count, so the last block's exchange
// (issued after its count saw every other block's) finds every OR.  The
// acq_rel fences this replaced cost an L2 write-back and an L1 invalidate
// each (buffer_wbl2 / buffer_inv sc1), four and three of them on the
// critical block's tail.
COA_DEV void lat_block_done(const CertArgs& a, uint32_t c, uint32_t bits) {
  if (bits) (void)__hip_atomic_fetch_or(a.status + c, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (!a.host_res) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const uint32_t old = __hip_atomic_fetch_add(a.done_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (old + 1 != a.total_blocks) return;
  HDR_MARK(6)
  __hip_atomic_store(a.done_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (uint32_t k = 0; k < a.nc; k++) {
    const uint32_t st = __hip_atomic_exchange(a.status + k, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(a.host_res + k, (a.tag << 8) | (st & 0xffu), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

COA_DEV void cert_lat_body(const CertArgs& a) {
  const uint32_t wave = coa_sha::uni(threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63;
  if (blockIdx.x < a.nc) {  // header digest: schedule in parallel, rounds on wave 0
    __shared__ uint64_t kw_lds[KW_CHUNK * 80];
    const uint32_t c = blockIdx.x;
    if (c == 0 && threadIdx.x == 0) { HDR_MARK(0) }
    const uint64_t o0 = uni64(a.hdr_off[c]), len = uni64(a.hdr_off[c + 1]) - o0;
    if (c == 0 && threadIdx.x == 0 && len != ~0ull) { HDR_MARK(4) }
    const uint8_t* p = a.hdr_data + o0;
    const uint64_t nblk = (len + 17 + 127) / 128;
    // the rounds on wave 0, each lane pair running one round's two halves
    // (coa_sha512.h, compress_kw2); lane 0 ends with the whole state
    const coa_sha::Lane2 L2 = coa_sha::lane2(lane);
    uint64_t hs[4];
    coa_sha::init2(hs, L2);
#pragma unroll 1
    for (uint64_t b0 = 0; b0 < nblk; b0 += KW_CHUNK) {
      const uint32_t nb = (uint32_t)min<uint64_t>(KW_CHUNK, nblk - b0);
      if (threadIdx.x < nb) {
        uint64_t W[16];
        coa_sha::padded_block(W, p, len, b0 + threadIdx.x, nblk);
        if (c == 0 && threadIdx.x == 0 && b0 == 0 && W[0] != 0x0123456789abcdefull) { HDR_MARK(8) }
        coa_sha::expand_kw(kw_lds + threadIdx.x * 80, W);
#ifdef COA_LAT_TRACE
        if (c == 0 && threadIdx.x == 0 && b0 == 0) {
          __builtin_amdgcn_s_waitcnt(0);  // the schedule's LDS writes done
          HDR_MARK(9)
        }
#endif
      }
      __syncthreads();
      if (c == 0 && threadIdx.x == 0 && b0 == 0) { HDR_MARK(1) }
      if (wave == 0) {
#pragma unroll 1
        for (uint32_t b = 0; b < nb; b++) coa_sha::compress_kw2(hs, kw_lds + b * 80, L2);
      }
      __syncthreads();
    }
    if (c == 0 && threadIdx.x == 0) { HDR_MARK(2) }
    if (wave) return;
    uint64_t st[8];
    coa_sha::gather2(st, hs);
    uint32_t h[16], id[8];
    coa_sha::state_to_le_words(h, st);
    load8u(id, a.ids + (uint64_t)c * 8);
    bool same = true;
#pragma unroll
    for (int i = 0; i < 8; i++) same = same && h[i] == id[i];
    if (c == 0 && lane == 0) { HDR_MARK(3) }
    if (lane == 0) lat_block_done(a, c, same ? 0u : (uint32_t)COA_CST_BAD_HEADER_ID);
    return;
  }
  __shared__ uint32_t s_lds[32];  // [s]B from wave 2
  __shared__ uint32_t s_ready;    // wave 2 published [s]B
  __shared__ rcmp::Shared cmp;    // wave 0's half of the compare, for wave 1
  if (threadIdx.x == 0) {
    s_ready = 0;
    cmp.ready = 0;
  }
  __syncthreads();
  const uint32_t job = blockIdx.x - a.nc;
  const bool hdr = job < a.nc;
  const uint32_t vi = job - a.nc;
  const uint32_t c = hdr ? job : vote_cert_u(a.voff, a.nc, vi);
  const uint32_t* sig = sel_ptr(hdr, a.hsigs + (uint64_t)c * 16, a.vsigs + (uint64_t)vi * 16);
  uint32_t rw[8];
  load8u(rw, sig);
  LAT_MARK(wave, 0)
  if (job == 0 && threadIdx.x == 0) { HDR_MARK(7) }
  if (wave == 1) {  // R's decompression on the wave's DPP rows, the compare, the verdict
    uint32_t bits = 0;
    const uint32_t res = rcmp::decompress_eq(cmp, rw, bits, [&] { LAT_MARK(1, 1) });
    LAT_MARK(1, 2)
    if (!(bits & COA_CST_UNCACHED)) {
      const uint32_t pre = bits >> 8;
      const bool r_ok = (res & 1u) != 0, eq = (res & 2u) != 0, small_r = (pre & 16) != 0;
      const bool s_ok = !(pre & 1), a_ok = !(pre & 2), small_a = (pre & 4) != 0, tfree = !(pre & 8);
      if (hdr) {
        bits = (s_ok && a_ok && r_ok && !small_a && !small_r && eq) ? 0u : COA_CST_BAD_HEADER_SIG;
      } else if (!(s_ok && a_ok && r_ok)) {
        bits = COA_CST_BAD_VOTES;
      } else {
        bits = (eq && tfree) ? 0u : COA_CST_VOTES_INCONCLUSIVE;
      }
    }
    LAT_MARK(1, 5)
    if (job == 0 && lane == 0) { HDR_MARK(5) }
    if (lane == 0) lat_block_done(a, c, bits);
    return;
  }
  // one comb term per lane (lanes 0..31; the upper half sums a copy),
  // [s]B on wave 2 from B's comb, [k](-A) on wave 0 from the key's comb
  uint32_t bits = 0;
  uint32_t dg[8];
  const uint32_t* tab = a.comb;
  int slot = 0;
  uint32_t pre = 0;
  if (wave == 2) {
    load8u(dg, sig + 8);
  } else {
    uint32_t pk[8], sw[8], msg[8];
    load8u(pk, sel_ptr(hdr, a.origins + (uint64_t)c * 8, a.vpks + (uint64_t)vi * 8));
    load8u(sw, sig + 8);
    load8u(msg, a.ids + (uint64_t)c * 8);
    slot = key_lookup_u(a.keys, a.nk, pk);
    if (slot < 0) {
      bits = COA_CST_UNCACHED;
      slot = 0;
    } else {
      uint64_t st[8];
      uint32_t h[16];
      if (!hdr) {  // Certificate::digest on the scalar unit
        uint32_t in[18];
        const uint64_t rd = uni64(a.rounds[c]);
#pragma unroll
        for (int i = 0; i < 8; i++) in[i] = msg[i];
        in[8] = (uint32_t)rd;
        in[9] = (uint32_t)(rd >> 32);
        load8u(in + 10, a.origins + (uint64_t)c * 8);
        coa_sha::hash_words<18>(st, in);
        coa_sha::state_to_le_words(h, st);
#pragma unroll
        for (int i = 0; i < 8; i++) msg[i] = h[i];
      }
      uint32_t in[24];
#pragma unroll
      for (int i = 0; i < 8; i++) {
        in[i] = rw[i];
        in[8 + i] = pk[i];
        in[16 + i] = msg[i];
      }
      coa_sha::hash_words<24>(st, in);
      coa_sha::state_to_le_words(h, st);
      sc k;
      sc_reduce512(k, h);
      const uint32_t kf = coa_sha::uni(a.kflags[slot]);
      const bool s_ok = sc_is_canonical(sw);
      const bool a_ok = (kf & COA_KEY_DECOMPRESSES) != 0;
      pre = (s_ok ? 0u : 1u) | (a_ok ? 0u : 2u) | ((kf & COA_KEY_SMALL_ORDER) ? 4u : 0u) |
            ((kf & COA_KEY_TORSION_FREE) ? 0u : 8u);
#pragma unroll
      for (int i = 0; i < 8; i++) dg[i] = k.v[i];
      tab = a.ktabs + (uint64_t)slot * COA_KEY_TAB_DWORDS;
    }
  }
  LAT_MARK(wave, 1)
  if (bits & COA_CST_UNCACHED) {  // wave 0 only: nothing to compare
    rcmp::skip(cmp, bits, lane == 0);
    return;
  }
  rp::P1 P;  // row form (coa_ge_rows.h)
  rcmp::comb_sum_rows(P, dg, tab, lane);
  LAT_MARK(wave, 3)
  if (wave == 2) {
    if (lane < 8) {
      s_lds[lane] = P.X;
      s_lds[8 + lane] = P.Y;
      s_lds[16 + lane] = P.Z;
      s_lds[24 + lane] = P.T;
    }
    if (lane == 0) __hip_atomic_store(&s_ready, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    return;
  }
  // wave 0: everything that needs only P while wave 1 is still decompressing
  // R (the critical chain): P = [s]B + [k](-A) as soon as wave 2 has
  // published [s]B, verify_strict's small-order test of R taken on P (an
  // accepting verdict needs R == P; headers only), the compare's P half
#pragma unroll 1
  while (__hip_atomic_load(&s_ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u)
    __builtin_amdgcn_s_sleep(1);
  rp::P1 S;
  S.X = rp::ld(s_lds);
  S.Y = rp::ld(s_lds + 8);
  S.Z = rp::ld(s_lds + 16);
  S.T = rp::ld(s_lds + 24);
  rcmp::add_rows(P, P, S);
  rcmp::prepare_rows(cmp, P, rw, pre << 8, hdr ? (16u << 8) : 0u, lane == 0);
  LAT_MARK(0, 4)
}

__global__ void __launch_bounds__(192) k_cert_verify_lat(CertArgs a) { cert_lat_body(a); }

// The same with the certificate's arrays read from the kernel arguments.  The
// buffer is addressed through the kernarg segment pointer (ci is the only
// argument, at offset 0): a pointer taken from the by-value parameter itself
// would make hipcc copy the whole 3 KB argument into scratch per thread.
__global__ void __launch_bounds__(192) k_cert_verify_lat_inl(CertInl ci) {
  CertArgs a = ci.a;
  const uint8_t* b = reinterpret_cast<const uint8_t*>(
                         reinterpret_cast<uintptr_t>(__builtin_amdgcn_kernarg_segment_ptr())) +
                     offsetof(CertInl, buf);
  a.hdr_data = b + ci.off_hdr;
  a.hdr_off = reinterpret_cast<const uint64_t*>(b + ci.off_hoff);
  a.ids = reinterpret_cast<const uint32_t*>(b + ci.off_ids);
  a.origins = reinterpret_cast<const uint32_t*>(b + ci.off_origins);
  a.hsigs = reinterpret_cast<const uint32_t*>(b + ci.off_hsigs);
  a.rounds = reinterpret_cast<const uint64_t*>(b + ci.off_rounds);
  a.voff = reinterpret_cast<const uint64_t*>(b + ci.off_voff);
  a.vpks = reinterpret_cast<const uint32_t*>(b + ci.off_vpks);
  a.vsigs = reinterpret_cast<const uint32_t*>(b + ci.off_vsigs);
  cert_lat_body(a);
}

// ---------------------------------------------------------------------------
// Grid of the throughput kernel: two waves per SIMD (256 CUs x 4 SIMDs x 2
// x 64 lanes), or one lane per job when there are fewer jobs.
// COA_CERT_LANES_TOTAL overrides (A/B runs).
// COA_CERT_WAVES=3: three waves per SIMD (the 168-VGPR instance, A/B).
static int cert_tp_waves() {
  const char* e = getenv("COA_CERT_WAVES");
  return (e && atoi(e) == 3) ? 3 : 2;
}

uint64_t cert_tp_lanes(uint64_t jobs) {
  uint64_t target = 256ull * 4 * (uint64_t)cert_tp_waves() * 64;
  if (const char* e = getenv("COA_CERT_LANES_TOTAL")) target = strtoull(e, nullptr, 10);
  if (target < 256) target = 256;
  const uint64_t lanes = jobs < target ? jobs : target;
  return (lanes + 255) / 256 * 256;
}

hipError_t coa_launch_key_flags(const uint32_t* keys, uint32_t nk, uint32_t* flags, hipStream_t s) {
  if (nk == 0) return hipSuccess;
  hipLaunchKernelGGL(k_key_flags, dim3((nk + 255) / 256), dim3(256), 0, s, keys, nk, flags);
  return hipGetLastError();
}

// Wide comb entry (key, j, m-1) = m * 2^(16 j) * (-A): with m = lo + 256 hi,
// lo a signed byte, it is the sum of the exact radix-256 comb entries
// (2j, lo) and (2j+1, hi) -- an integer multiple, torsion kept -- made affine.
__global__ void __launch_bounds__(256) k_key_wcomb(const uint32_t* __restrict__ tabs, uint32_t nk,
                                                   uint32_t* __restrict__ wtabs) {
  // grid-stride (a bounded, resident grid: see coa_launch_key_wcombs20)
  for (uint64_t id = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; id < (uint64_t)nk * COA_KWCOMB_ENTRIES;
       id += (uint64_t)gridDim.x * blockDim.x) {
  const uint32_t key = (uint32_t)(id / COA_KWCOMB_ENTRIES);
  const uint32_t e = (uint32_t)(id % COA_KWCOMB_ENTRIES);
  const int j = (int)(e >> (COA_KWCOMB_W - 1));
  const int m = (int)(e & ((1u << (COA_KWCOMB_W - 1)) - 1)) + 1;
  int lo = m & 255, hi = m >> 8;
  if (lo >= 128) {
    lo -= 256;
    hi += 1;
  }
  const uint32_t* ktab = tabs + (uint64_t)key * COA_KEY_TAB_DWORDS;
  ge_p3 P;
  ge_p3_identity(P);
  ge_p1p1 t;
  ge_niels q;
  comb_select(q, ktab, 2 * j, lo);
  ge_madd(t, P, q);
  ge_p1p1_to_p3(P, t);
  comb_select(q, ktab, 2 * j + 1, hi);
  ge_madd(t, P, q);
  ge_p1p1_to_p3(P, t);
  store_niels(wtabs + (uint64_t)key * COA_KWCOMB_DWORDS + (uint64_t)e * COA_KWC_STRIDE, P);
  }
}

// Widest comb entry (key, j, m-1) = m * 2^(20 j) * (-A): 20 j = 8 q + r, and
// m 2^r < 2^24 is recoded into signed bytes b0, b1, b2, so the entry is the
// sum of the exact radix-256 comb entries (q, b0), (q+1, b1), (q+2, b2) -- an
// integer multiple, torsion kept -- made affine.  At j = 12 (q = 30) a byte
// at position 32 would be needed only for m > 2^16, which no scalar below l
// produces (its top digit is at most 2^13, wc_recode): those entries are
// never read and hold the sum of the first two bytes.
__global__ void __launch_bounds__(256) k_key_wcomb20(const uint32_t* __restrict__ tabs, uint32_t nk,
                                                     uint32_t* __restrict__ wtabs) {
  // grid-stride (a bounded, resident grid: see coa_launch_key_wcombs20)
  for (uint64_t id = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; id < (uint64_t)nk * COA_KWCOMB20_ENTRIES;
       id += (uint64_t)gridDim.x * blockDim.x) {
  const uint32_t key = (uint32_t)(id / COA_KWCOMB20_ENTRIES);
  const uint64_t e = id % COA_KWCOMB20_ENTRIES;
  const int j = (int)(e >> (COA_KWCOMB20_W - 1));
  const uint32_t m = (uint32_t)(e & ((1u << (COA_KWCOMB20_W - 1)) - 1)) + 1;
  const int bit = COA_KWCOMB20_W * j, q = bit >> 3;
  uint32_t v = m << (bit & 7);
  int b[3];
  int carry = 0;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    int x = (int)(v & 255u) + carry;
    v >>= 8;
    carry = 0;
    if (i < 2 && x >= 128) {
      x -= 256;
      carry = 1;
    }
    b[i] = x;
  }
  const uint32_t* ktab = tabs + (uint64_t)key * COA_KEY_TAB_DWORDS;
  ge_p3 P;
  ge_p3_identity(P);
  ge_p1p1 t;
  ge_niels qn;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    if (q + i > 31) break;
    comb_select(qn, ktab, q + i, b[i]);
    ge_madd(t, P, qn);
    ge_p1p1_to_p3(P, t);
  }
  store_niels(wtabs + (uint64_t)key * COA_KWCOMB20_DWORDS + e * COA_KWC_STRIDE, P);
  }
}

// The wide key combs are built while the device serves live windows (a
// registration builds the next key-cache generation beside the current one,
// on a least-priority stream: coa_runtime.cpp build_keyset).  One workgroup
// per 256 entries by default -- short workgroups, so the scheduler hands the
// CUs to the windows' workgroups between them; COA_BUILD_BLOCKS=<n> bounds
// the grid to n resident workgroups striding over the entries (A/B:
// slower build, p99 0.65 vs 0.89 ms under a 5,000/s certificate stream).
static uint32_t build_blocks(uint64_t total) {
  const char* e = getenv("COA_BUILD_BLOCKS");
  const uint64_t cap = e ? strtoull(e, nullptr, 10) : 0;
  const uint64_t want = (total + 255) / 256;
  return (uint32_t)(want < cap ? want : (cap ? cap : want));
}

hipError_t coa_launch_key_wcombs20(const uint32_t* tabs, uint32_t nk, uint32_t* wtabs, hipStream_t s) {
  if (nk == 0) return hipSuccess;
  const uint64_t total = (uint64_t)nk * COA_KWCOMB20_ENTRIES;
  hipLaunchKernelGGL(k_key_wcomb20, dim3(build_blocks(total)), dim3(256), 0, s, tabs, nk, wtabs);
  return hipGetLastError();
}

hipError_t coa_launch_key_wcombs(const uint32_t* tabs, uint32_t nk, uint32_t* wtabs, hipStream_t s) {
  if (nk == 0) return hipSuccess;
  const uint64_t total = (uint64_t)nk * COA_KWCOMB_ENTRIES;
  hipLaunchKernelGGL(k_key_wcomb, dim3(build_blocks(total)), dim3(256), 0, s, tabs, nk, wtabs);
  return hipGetLastError();
}

hipError_t coa_launch_key_tables(const uint32_t* keys, uint32_t nk, uint32_t* tabs, hipStream_t s) {
  if (nk == 0) return hipSuccess;
  const uint64_t lanes = (uint64_t)nk * COA_KEY_TAB_ENTRIES;
  hipLaunchKernelGGL(k_key_tables, dim3((uint32_t)((lanes + 255) / 256)), dim3(256), 0, s, keys, nk, tabs);
  return hipGetLastError();
}

hipError_t coa_launch_cert_verify_inl(const CertInl& ci, hipStream_t s) {
  if (ci.a.nc == 0) return hipSuccess;
  CertInl c = ci;
  c.a.hdr_blocks = (c.a.nc + 255) / 256;
  const uint32_t jobs = c.a.nc + c.a.nv;
  c.a.total_blocks = c.a.nc + jobs;
  hipLaunchKernelGGL(k_cert_verify_lat_inl, dim3(c.a.total_blocks), dim3(192), 0, s, c);
  return hipGetLastError();
}

// Jobs in key order for the throughput kernel.  A chunk of 64 consecutive
// jobs in certificate order holds 64 different keys (a certificate's votes
// come from distinct members), so each of the 13 key-comb additions reads 64
// random entries of 64 different 654 MB combs: half the kernel's requests
// missed the per-CU translation cache (profiles/r05_cert_tlb_pmc.txt).  Sorted
// by key slot, a chunk's lanes read one key's comb.  A counting sort with
// few contended atomics (one global counter per key took 680k of them,
// 0.4 ms): COA_SORT_WGS workgroups each count a contiguous range of jobs
// per slot in LDS (unregistered keys in the last bin), keep the counts
// (counts[wg][bin]) and add them to the bin totals (one atomic per
// workgroup and bin); one block turns the totals into start cursors; each
// workgroup then reserves its range in every bin it uses (one atomic each)
// and places its jobs with LDS counters.  The order inside a bin is
// arbitrary: every job's verdict depends on its own inputs only.
#define COA_SORT_BINS 4096
#define COA_SORT_WGS 256
// smallest call the key-order sort pays for (its three launches)
#define COA_SORT_MIN_JOBS 16384
__global__ void __launch_bounds__(256) k_job_count(CertArgs a, uint32_t bins, uint32_t per,
                                                   uint32_t* __restrict__ total, uint32_t* __restrict__ counts,
                                                   uint32_t* __restrict__ bin) {
  __shared__ uint32_t h[COA_SORT_BINS];
  for (uint32_t k = threadIdx.x; k < bins; k += blockDim.x) h[k] = 0;
  __syncthreads();
  const uint64_t jobs = (uint64_t)a.nc + a.nv;
  const uint64_t lo = (uint64_t)blockIdx.x * per, hi = lo + per < jobs ? lo + per : jobs;
  for (uint64_t j = lo + threadIdx.x; j < hi; j += blockDim.x) {
    uint32_t pk[8];
    load8(pk, j < a.nc ? a.origins + j * 8 : a.vpks + (j - a.nc) * 8);
    const int slot = key_lookup(a.keys, a.nk, pk);
    const uint32_t b = slot < 0 ? a.nk : (uint32_t)slot;
    bin[j] = b;
    atomicAdd(h + b, 1u);
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < bins; k += blockDim.x) {
    const uint32_t c = h[k];
    counts[(uint64_t)blockIdx.x * COA_SORT_BINS + k] = c;
    if (c) atomicAdd(total + k, c);
  }
}
// Bin totals -> exclusive start cursors, in place, one block.
__global__ void __launch_bounds__(1024) k_job_scan(uint32_t* __restrict__ v, uint32_t n) {
  __shared__ uint32_t part[1024];
  const uint32_t t = threadIdx.x, per = (n + 1023) / 1024;
  uint32_t mine[COA_SORT_BINS / 1024], sum = 0;
#pragma unroll
  for (uint32_t i = 0; i < COA_SORT_BINS / 1024; i++) {
    const uint32_t k = t * per + i;
    mine[i] = (i < per && k < n) ? v[k] : 0u;
    sum += mine[i];
  }
  part[t] = sum;
  __syncthreads();
  for (uint32_t o = 1; o < 1024; o <<= 1) {  // inclusive scan of the per-thread sums
    const uint32_t x = t >= o ? part[t - o] : 0u;
    __syncthreads();
    part[t] += x;
    __syncthreads();
  }
  uint32_t run = part[t] - sum;  // exclusive start of this thread's bins
#pragma unroll
  for (uint32_t i = 0; i < COA_SORT_BINS / 1024; i++) {
    const uint32_t k = t * per + i;
    if (i < per && k < n) v[k] = run;
    run += mine[i];
  }
}
__global__ void __launch_bounds__(256) k_job_place(uint64_t jobs, uint32_t bins, uint32_t per,
                                                   uint32_t* __restrict__ cursor, const uint32_t* __restrict__ counts,
                                                   const uint32_t* __restrict__ bin, uint32_t* __restrict__ perm) {
  __shared__ uint32_t cur[COA_SORT_BINS];
  for (uint32_t k = threadIdx.x; k < bins; k += blockDim.x) {
    const uint32_t c = counts[(uint64_t)blockIdx.x * COA_SORT_BINS + k];
    cur[k] = c ? atomicAdd(cursor + k, c) : 0u;  // this workgroup's range in bin k
  }
  __syncthreads();
  const uint64_t lo = (uint64_t)blockIdx.x * per, hi = lo + per < jobs ? lo + per : jobs;
  for (uint64_t j = lo + threadIdx.x; j < hi; j += blockDim.x) perm[atomicAdd(cur + bin[j], 1u)] = (uint32_t)j;
}

// Signature chunks one wave of the throughput grid may take (its slab
// capacity): the even share plus slack for the waves that run ahead.
static uint32_t cert_tp_jcap(uint64_t jobs, uint64_t lanes) {
  const uint64_t waves = lanes / 64, chunks = (jobs + 63) / 64;
  return (uint32_t)((chunks + waves - 1) / waves + 2);
}

// Throughput scratch: [0, 256) chunk counter | slab (lanes x jcap jobs) |
// Certificate::digest per certificate (at most one per job).
static size_t cert_slab_bytes(uint64_t jobs, uint64_t lanes) {
  return (size_t)(lanes * cert_tp_jcap(jobs, lanes) * PSCR_ROWS * 16);
}

// ... | key-order sort, only for a call that may sort (key_order and at
// least COA_SORT_MIN_JOBS jobs): bin totals / cursors [COA_SORT_BINS], counts
// [COA_SORT_WGS][COA_SORT_BINS], each job's bin [jobs], the permutation [jobs]
// (~4.2 MB + 8 B per job; a latency, pipelined-chunk or queue workspace does
// not carry it)
size_t coa_cert_scratch_bytes(uint64_t jobs, bool key_order) {
  const uint64_t lanes = cert_tp_lanes(jobs ? jobs : 1);
  const size_t base = 256 + cert_slab_bytes(jobs, lanes) + (size_t)(jobs ? jobs : 1) * 32;
  if (!key_order || jobs < COA_SORT_MIN_JOBS) return base;
  return base + 256 + (size_t)COA_SORT_BINS * (COA_SORT_WGS + 1) * 4 + (size_t)jobs * 8;
}

hipError_t coa_launch_cert_verify(CertArgs a, int lanes_per_sig, uint32_t* pscr, hipStream_t s) {
  if (a.nc == 0) return hipSuccess;
  a.hdr_blocks = (a.nc + 255) / 256;
  const uint64_t jobs = (uint64_t)a.nc + a.nv;
  if (lanes_per_sig == 64) {  // one workgroup per header digest and per signature
    a.total_blocks = (uint32_t)(a.nc + jobs);
    hipLaunchKernelGGL(k_cert_verify_lat, dim3((uint32_t)(a.nc + jobs)), dim3(192), 0, s, a);
    return hipGetLastError();
  }
  const uint64_t lanes = cert_tp_lanes(jobs);
  // the chunk counter (pscr[0]) starts at zero; the slab follows it, then the
  // certificates' digests (prologue kernel)
  hipError_t e = hipMemsetAsync(pscr, 0, 4, s);
  if (e != hipSuccess) return e;
  // the prologue pays for its launch when certificates carry many votes (C3:
  // 67 votes, +2-5 %); with few (C1: 3 votes) the digest stays per vote.
  // COA_CERT_DIGEST_PER_VOTE=1 forces per vote (A/B).
  if (a.nv >= 8ull * a.nc && !getenv("COA_CERT_DIGEST_PER_VOTE")) {
    uint32_t* cdig = pscr + 64 + cert_slab_bytes(jobs, lanes) / 4;
    hipLaunchKernelGGL(k_cert_digests, dim3((a.nc + 255) / 256), dim3(256), 0, s, a, cdig);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    a.cdig = cdig;
  }
  // jobs in key order when the caller asks for it, the committee fits the
  // bins and the call is large enough to pay for the sort
  // (COA_CERT_KEYSORT=0: certificate order everywhere, A/B).  The callers
  // that ask: the device-resident round (+16-18 %); not the pipelined host
  // chunks nor the queue's windows, whose concurrent launches lost more to
  // the sort's own launches than the order gained (profiles/r05_cert_keysort_ab.txt)
  const char* ks = getenv("COA_CERT_KEYSORT");
  if (a.key_order && a.nk > 0 && a.nk + 1 <= COA_SORT_BINS && jobs >= COA_SORT_MIN_JOBS &&
      !(ks && ks[0] == '0' && ks[1] == 0)) {
    uint32_t* total = pscr + 64 + cert_slab_bytes(jobs, lanes) / 4 + (size_t)jobs * 8 + 64;
    uint32_t* counts = total + COA_SORT_BINS;
    uint32_t* bin = counts + (size_t)COA_SORT_BINS * COA_SORT_WGS;
    uint32_t* perm = bin + jobs;
    const uint32_t bins = a.nk + 1, per = (uint32_t)((jobs + COA_SORT_WGS - 1) / COA_SORT_WGS);
    e = hipMemsetAsync(total, 0, bins * 4, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_job_count, dim3(COA_SORT_WGS), dim3(256), 0, s, a, bins, per, total, counts, bin);
    hipLaunchKernelGGL(k_job_scan, dim3(1), dim3(1024), 0, s, total, bins);
    hipLaunchKernelGGL(k_job_place, dim3(COA_SORT_WGS), dim3(256), 0, s, jobs, bins, per, total, counts, bin, perm);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    a.perm = perm;
  }
  if (cert_tp_waves() == 3)
    hipLaunchKernelGGL(k_cert_verify<3>, dim3((uint32_t)(a.hdr_blocks + lanes / 256)), dim3(256), 0, s, a, pscr,
                       cert_tp_jcap(jobs, lanes));
  else
    hipLaunchKernelGGL(k_cert_verify<2>, dim3((uint32_t)(a.hdr_blocks + lanes / 256)), dim3(256), 0, s, a, pscr,
                       cert_tp_jcap(jobs, lanes));
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// coa_fe_rows_check: the row-parallel chains against the one-lane ones.
__global__ void __launch_bounds__(64) k_fe_rows_check(const uint8_t* __restrict__ in, uint32_t n,
                                                      uint32_t* __restrict__ out) {
  const uint32_t i = blockIdx.x;
  uint32_t w[8], w2[8];
  load8u(w, reinterpret_cast<const uint32_t*>(in + (uint64_t)i * 32));
  load8u(w2, reinterpret_cast<const uint32_t*>(in + (uint64_t)((i + 1) % n) * 32));
  fe x, y;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    x.v[k] = w[k];
    y.v[k] = w2[k];
  }
  uint32_t bad = 0;
  fe a, b;
  fe_pow_p58_rows(a, x);
  fe_pow_p58(b, x);
  bad |= fe_eq(a, b) ? 0u : 1u;
  fe_invert_rows(a, x);
  fe_invert(b, x);
  bad |= fe_eq(a, b) ? 0u : 2u;
  fw::to_fe(a, fw::mul(fw::from_fe(x), fw::from_fe(y)));
  fe_mul(b, x, y);
  bad |= fe_eq(a, b) ? 0u : 4u;
  fw::to_fe(a, fw::add(fw::from_fe(x), fw::from_fe(y)));
  fe_add(b, x, y);
  bad |= fe_eq(a, b) ? 0u : 16u;
  fw::to_fe(a, fw::sub(fw::from_fe(x), fw::from_fe(y)));
  fe_sub(b, x, y);
  bad |= fe_eq(a, b) ? 0u : 32u;
  ge_p3 P, Q;
  const bool ok_r = ge_decompress<true>(P, w);
  const bool ok_s = ge_decompress(Q, w);
  if (ok_r != ok_s || (ok_s && !(fe_eq(P.X, Q.X) && fe_eq(P.Y, Q.Y) && fe_eq(P.T, Q.T)))) bad |= 8u;
  if (threadIdx.x == 0) out[i] = bad;
}

hipError_t coa_launch_fe_rows_check(const uint8_t* in, uint32_t n, uint32_t* out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_fe_rows_check, dim3(n), dim3(64), 0, s, in, n, out);
  return hipGetLastError();
}
