// Internal launch wrappers for the halved-scalar verification path
// (coa_halved.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// wide HBM comb of B (coa_smul.h): positions x magnitudes, 24 dwords each
// (overridable for A/B builds, tools/build_variant.py: W = 26 with 10
// positions is a 32 GB comb)
#ifndef COA_WCOMB_W
#define COA_WCOMB_W 24
#define COA_WCOMB_POS 11
#endif
#define COA_WCOMB_MAG (1u << (COA_WCOMB_W - 1))
#define COA_WCOMB_ENTRIES ((uint64_t)COA_WCOMB_POS * COA_WCOMB_MAG)
// Dwords per entry of B's wide comb: the entry's 24 (y+x, y-x, 2dxy) plus 8
// of padding, so an entry is one 128-byte line.  At 24 an entry at a random
// index straddles two lines half the time: 1.5 lines (192 B) fetched per 96 B
// used.  Same-box A/B (profiles/r06_stride_ab.txt): C2 +0.2-0.65 % in three
// of three pairs for 3 GB more (11.9 GB); the keys' combs gained nothing on
// the C3 round (VALU-bound, DESIGN.md §4 "C3 roofline") and keep 24
// (COA_KWC_STRIDE, coa_committee.h).  -DCOA_WC_STRIDE=24: the round-5 layout.
#ifndef COA_WC_STRIDE
#define COA_WC_STRIDE 32
#endif
#define COA_WCOMB_DWORDS (COA_WCOMB_ENTRIES * COA_WC_STRIDE)
#define COA_COMB_ENTRIES (32 * 128)
#define COA_COMB_DWORDS (COA_COMB_ENTRIES * 24)
// k_halve record per signature: c[8] | |d|[8] | e[8] | meta | pad[7]
#define COA_HALVE_REC_BYTES 128
// per-lane scratch of k_verify_halved: j*(-A) and j*(-/+R), 8 entries each
#define COA_HALVED_SCRATCH_PER_LANE 2048

hipError_t coa_launch_build_comb(uint32_t* comb, const uint32_t* btab, hipStream_t s);
hipError_t coa_launch_halve(const uint32_t* kbuf, const uint8_t* sigs, uint32_t n, uint32_t* rec, hipStream_t s);
hipError_t coa_launch_verify_halved(const uint8_t* pks, const uint8_t* sigs, const uint32_t* rec, uint32_t n,
                                    uint8_t* verdicts, uint32_t* scratch, uint32_t scratch_lanes,
                                    const uint32_t* comb, const uint32_t* wcomb, int waves, hipStream_t s);
// Items per launch pair of the split path (one 2 KiB slab each: 4 GiB of HBM
// at 2^21, i.e. eight waves per SIMD in k_verify_main).
#define COA_SPLIT_CHUNK (1u << 21)
// Split verification of n <= COA_SPLIT_CHUNK items: k_pre_halve
// (decompressions + slab tables, and k + halving + [e]B, in one two-role
// launch) then k_verify_main.  k comes from kbuf, or is hashed in-kernel from
// msgs (msg_len bytes per item, contiguous) when msgs is non-null.
// flags: n bytes; scratch: n slabs of COA_HALVED_SCRATCH_PER_LANE bytes;
// ebp: n x 128 bytes to compute [e]B in phase 1, or null for phase 2.
hipError_t coa_launch_verify_split(const uint8_t* pks, const uint8_t* sigs, const uint8_t* msgs, uint32_t msg_len,
                                   const uint32_t* kbuf, uint32_t n, uint32_t* rec, uint8_t* flags,
                                   uint8_t* verdicts, uint32_t* scratch, uint32_t* ebp, const uint32_t* comb,
                                   const uint32_t* wcomb, hipStream_t s);
// wide HBM comb of B (coa_smul.h, COA_WCOMB_*): build from the radix-256
// comb, and the whole-table consistency check (count of bad entries in *bad,
// zeroed by the caller)
hipError_t coa_launch_build_wcomb(uint32_t* wcomb, const uint32_t* comb, hipStream_t s);
hipError_t coa_launch_check_wcomb(const uint32_t* wcomb, uint32_t* bad, hipStream_t s);
