// Internal launch wrappers between the HIP kernels (coa_kernels.hip) and the
// host runtime / C ABI (coa_runtime.cpp).  Not part of the public ABI
// (that is include/coa_verify.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define COA_VERIFY_BLOCK 256
#define COA_BTAB_DWORDS (128 * 24)
// lanes of the verify grid (each holds a 1 KiB j·(-A) table in the scratch slab)
#define COA_VERIFY_MAX_LANES (256 * 4 * 256)

hipError_t coa_launch_build_btable(uint32_t* tab, hipStream_t s);
hipError_t coa_launch_hram(const uint8_t* msgs, uint32_t msg_len, uint64_t msg_stride, const uint32_t* msg_index,
                           const uint8_t* pks, const uint8_t* sigs, uint32_t n, uint32_t* k_out, hipStream_t s);
hipError_t coa_launch_verify_strict(const uint8_t* pks, const uint8_t* sigs, const uint32_t* k_in, uint32_t n,
                                    uint8_t* verdicts, uint32_t* scratch, uint32_t scratch_lanes,
                                    const uint32_t* btab, hipStream_t s);
hipError_t coa_launch_sha512_many(const uint8_t* data, const uint64_t* off, uint32_t n, uint32_t* out,
                                  hipStream_t s);
hipError_t coa_launch_keygen(const uint8_t* seeds, uint32_t n, uint8_t* pks, uint32_t* aux, const uint32_t* btab,
                             hipStream_t s);
hipError_t coa_launch_sign_r(const uint32_t* aux, const uint8_t* msgs, uint32_t msg_len, uint32_t n, uint8_t* sigs,
                             uint32_t* rbuf, const uint32_t* btab, hipStream_t s);
hipError_t coa_launch_sign_s(const uint32_t* aux, const uint32_t* rbuf, const uint32_t* kbuf, uint32_t n,
                             uint8_t* sigs, hipStream_t s);
