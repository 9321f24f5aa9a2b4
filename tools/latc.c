/* Latency of the drop-in's one-item entry points as a compiled caller sees
 * them: the Rust crate calls coa_certificate_verify / coa_ed25519_verify_strict
 * through its extern "C" binding (rust/crypto/src/coa_ffi.rs), with no
 * per-call argument marshalling.  bench.py times the same calls through the
 * Python test binding (ctypes + numpy conversions) as well; this loop takes
 * that binding out of the clock.  Each sample is one blocking call: host
 * pointers in, verdict out.
 *
 * Built by xrpl-coa-prototype_amd/build.py into lib/liblatc.so (gcc, linked
 * against libcoa_verify.so).  Measurement infrastructure only. */
#define _POSIX_C_SOURCE 199309L
#include <stddef.h>
#include <stdint.h>
#include <time.h>

#include "coa_verify.h"

static double now_us(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec * 1e6 + (double)t.tv_nsec * 1e-3;
}

/* `samples` calls of coa_certificate_verify on one certificate; per-call
 * microseconds into out_us.  Returns 0, or the first non-zero result. */
int latc_certificate(const uint8_t* header_data, size_t header_len, const uint8_t* id, const uint8_t* origin,
                     const uint8_t* header_sig, uint64_t round, const uint8_t* vote_pks, const uint8_t* vote_sigs,
                     size_t n_votes, int samples, double* out_us) {
  for (int i = 0; i < samples; i++) {
    const double t0 = now_us();
    const int rc = coa_certificate_verify(header_data, header_len, id, origin, header_sig, round, vote_pks, vote_sigs,
                                          n_votes, 0);
    out_us[i] = now_us() - t0;
    if (rc != 0) return rc;
  }
  return 0;
}

/* `samples` calls of coa_ed25519_verify_strict cycling over n triples
 * (32-byte messages); per-call microseconds into out_us. */
int latc_verify(const uint8_t* msgs, const uint8_t* pks, const uint8_t* sigs, int n, int samples, double* out_us) {
  for (int i = 0; i < samples; i++) {
    const int j = i % n;
    const double t0 = now_us();
    const int rc = coa_ed25519_verify_strict(msgs + 32 * j, pks + 32 * j, sigs + 64 * j);
    out_us[i] = now_us() - t0;
    if (rc != 0) return rc;
  }
  return 0;
}
