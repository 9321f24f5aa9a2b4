// Internal launch wrappers for the batch (RLC) verification kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// per-lane scratch of k_batch_terms: two 8-entry cached tables (2 KiB)
#define COA_BATCH_SCRATCH_PER_LANE 2048

// z_i binds (seed, group, i): group = group_of[i], or group_const when
// group_of is NULL (one group per launch)
hipError_t coa_launch_batch_z(const uint32_t* kbuf, const uint8_t* sigs, const uint32_t* group_of,
                              uint32_t group_const, uint32_t n, uint64_t seed, uint32_t* zs, hipStream_t s);
hipError_t coa_launch_batch_terms(const uint8_t* pks, const uint8_t* sigs, const uint32_t* kbuf, const uint32_t* zs,
                                  uint32_t n, uint32_t* terms, uint8_t* flags, uint32_t* scratch,
                                  uint32_t scratch_lanes, const uint32_t* btab, hipStream_t s);
hipError_t coa_launch_batch_reduce(const uint64_t* offs, uint32_t n_groups, const uint32_t* terms,
                                   const uint8_t* flags, uint8_t* verdicts, hipStream_t s);
