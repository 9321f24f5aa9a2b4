// Internal launch wrappers for the Pippenger batch-equation path
// (coa_msm.hip): Signature::verify_batch over one large group.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define COA_MSM_C 9                      // window bits (signed digits, |d| <= 256)
#define COA_MSM_NB 256                   // buckets per window
#define COA_MSM_WA 29                    // windows of a 253-bit scalar (A_i, B)
#define COA_MSM_WR 15                    // windows of a 128-bit weight z_i (R_i)
#define COA_MSM_RUN 64                   // max sorted entries per lane in k_msm_bucket
#define COA_MSM_CHUNK (256 * COA_MSM_RUN)  // points per bucket workgroup
#define COA_MSM_PREP_BLOCKS 1024         // k_msm_prep grid (partial sums of z_i s_i)

// Device workspace of one call over n signatures (np = 2n + 1 points).
struct MsmWs {
  uint32_t nchunks_cap;  // chunks the part/segs arrays hold
  uint32_t* k;     // n x 8   challenge scalars h_i
  uint32_t* z;     // n x 4   128-bit weights z_i
  uint32_t* pts;   // np x 24 Niels points: R_0..R_{n-1}, A_0..A_{n-1}, B
  int16_t* dig;    // WA x np signed digits, window-major
  uint32_t* zpart; // PREP_BLOCKS x 9  partial sums of z_i s_i mod l
  uint32_t* part;  // WA x nchunks x 32  per-(window, chunk) sums  sum_j j B_j
  uint32_t* wsum;  // WA x 32  per-window sums
  uint32_t* bad;   // 1: an encoding check failed
  uint32_t* segs;  // WA x nchunks x 512 x 32  bucket segments of k_msm_bucket
};
size_t coa_msm_ws_bytes(size_t n);
MsmWs coa_msm_ws_carve(void* base, size_t n);
uint32_t coa_msm_chunks(size_t n);

// k and z must already be in ws (k_hram, k_batch_z or caller-given weights).
hipError_t coa_launch_msm(const uint8_t* pks, const uint8_t* sigs, uint32_t n, const MsmWs& ws, uint8_t* verdict,
                          hipStream_t s);
