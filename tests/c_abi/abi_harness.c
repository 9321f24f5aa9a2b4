/* C harness of the engine's C ABI: compiled with gcc -std=c11 -Wall -Wextra
 * -Werror against include/coa_verify.h and linked against libcoa_verify.so,
 * so every prototype the header declares is checked by a C compiler (ctypes
 * checks only that the symbols exist).  It calls EVERY entry point once.
 *
 *   abi_harness cpu   no GPU: every call that needs the device must return
 *                     COA_ENODEVICE (no CPU fallback); host-only calls (wire
 *                     decode, sizes, version, argument checks) behave as on a
 *                     GPU box.
 *   abi_harness gpu   GPU box: the reference's "Hello, world!" signature
 *                     (crypto/src/tests/crypto_tests.rs:49-60) verifies Ok,
 *                     a corrupted copy Err, through every verify entry point.
 * Exit 0 = all checks passed; prints the first failing check otherwise. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "coa_verify.h"

static int failures = 0;
#define CHECK(cond, what)                                         \
  do {                                                            \
    if (!(cond)) {                                                \
      fprintf(stderr, "FAIL %s (line %d): %s\n", what, __LINE__, coa_last_error()); \
      failures++;                                                 \
    }                                                             \
  } while (0)

static void unhex(uint8_t* out, const char* hex, size_t n) {
  for (size_t i = 0; i < n; i++) {
    unsigned v = 0;
    sscanf(hex + 2 * i, "%2x", &v);
    out[i] = (uint8_t)v;
  }
}

static void cb(void* user, int status, const uint8_t* verdicts, size_t n) {
  int* seen = (int*)user;
  (void)verdicts;
  (void)n;
  *seen = status;
}

int main(int argc, char** argv) {
  const int gpu = argc > 1 && strcmp(argv[1], "gpu") == 0;
  const int dev_rc = gpu ? COA_OK : COA_ENODEVICE;
  uint8_t msg[32], pk[32], sig[64], bad[64];
  unhex(msg, "c1527cd893c124773d811911970c8fe6e857d6df5dc9226bd8a160614c0cd963", 32);
  unhex(pk, "beada06126c78d98b4a1a69f6ee6189694f0f4751538da824f1adc8b14a1b562", 32);
  unhex(sig,
        "fd1017091c871c5feb5b171ada10a5b636522f10ce6a2c8cbec12dafe78455a5"
        "693a194e5b7a3baa25fbd5b04dbfed62a3b766872435625f1d7aeeace9afcd07",
        64);
  memcpy(bad, sig, 64);
  bad[40] ^= 1;

  /* lifecycle */
  CHECK(coa_version() != NULL && strlen(coa_version()) > 0, "coa_version");
  CHECK(coa_init(0) == dev_rc, "coa_init");
  const int ids[1] = {0};
  CHECK(coa_init_devices(ids, 1) == dev_rc, "coa_init_devices");
  CHECK(coa_init_devices(NULL, 0) == COA_EINVAL, "coa_init_devices(empty)");
  const int ndev = coa_device_count();
  CHECK(gpu ? ndev >= 1 : ndev == COA_ENODEVICE, "coa_device_count");
  int idbuf[8] = {-1, -1, -1, -1, -1, -1, -1, -1};
  const int nids = coa_device_ids(idbuf, 8);
  CHECK(gpu ? (nids == ndev && idbuf[0] >= 0) : nids == COA_ENODEVICE, "coa_device_ids");
  uint64_t bad_entries = 7;
  CHECK(coa_self_test(0, &bad_entries) == dev_rc, "coa_self_test");
  CHECK(!gpu || bad_entries == 0, "coa_self_test entries");
  CHECK(coa_fe_rows_check_device(0, NULL, 0, NULL, NULL) == dev_rc, "coa_fe_rows_check_device");
  uint64_t rebuilt = 9, rerun = 9;
  CHECK(coa_engine_recoveries(&rebuilt, &rerun) == COA_OK && rebuilt == 0 && rerun == 0, "coa_engine_recoveries");

  /* Signature::verify */
  CHECK(coa_ed25519_verify_strict(msg, pk, sig) == (gpu ? COA_OK : COA_ENODEVICE), "verify_strict ok");
  CHECK(coa_ed25519_verify_strict(msg, pk, bad) == (gpu ? COA_REJECT : COA_ENODEVICE), "verify_strict bad");
  uint8_t msgs2[64], pks2[64], sigs2[128], v2[2] = {9, 9};
  memcpy(msgs2, msg, 32);
  memcpy(msgs2 + 32, msg, 32);
  memcpy(pks2, pk, 32);
  memcpy(pks2 + 32, pk, 32);
  memcpy(sigs2, sig, 64);
  memcpy(sigs2 + 64, bad, 64);
  CHECK(coa_ed25519_verify_strict_many(msgs2, 32, pks2, sigs2, 2, v2) == dev_rc, "verify_strict_many");
  CHECK(!gpu || (v2[0] == 0 && v2[1] == 1), "verify_strict_many verdicts");
  CHECK(coa_verify_workspace_bytes(1024) > 0, "coa_verify_workspace_bytes");
  CHECK(coa_ed25519_verify_strict_many_device(0, NULL, 32, NULL, NULL, 0, NULL, NULL, NULL) == dev_rc,
        "verify_strict_many_device(n=0)");
  CHECK(coa_ed25519_challenge_many_device(0, NULL, 32, NULL, NULL, 0, NULL, NULL) == dev_rc,
        "challenge_many_device(n=0)");
  CHECK(coa_ed25519_verify_prehashed_many_device(0, NULL, NULL, NULL, 0, NULL, NULL, NULL) == dev_rc,
        "verify_prehashed_many_device(n=0)");

  /* Signature::verify_batch */
  CHECK(coa_ed25519_verify_batch(msg, pk, sig, 1, 5) == (gpu ? COA_OK : COA_ENODEVICE), "verify_batch ok");
  CHECK(coa_ed25519_verify_batch(msg, pk, bad, 1, 5) == (gpu ? COA_REJECT : COA_ENODEVICE), "verify_batch bad");
  const uint64_t goff[3] = {0, 1, 2};
  uint8_t gv[2] = {9, 9};
  CHECK(coa_ed25519_verify_batch_groups(msgs2, pks2, sigs2, goff, 2, gv, 5) == dev_rc, "verify_batch_groups");
  CHECK(!gpu || (gv[0] == 0 && gv[1] == 1), "verify_batch_groups verdicts");
  uint8_t zs[32];
  memset(zs, 3, sizeof zs);
  CHECK(coa_ed25519_verify_batch_groups_z(msgs2, pks2, sigs2, goff, 2, zs, gv) == dev_rc, "verify_batch_groups_z");
  CHECK(!gpu || (gv[0] == 0 && gv[1] == 1), "verify_batch_groups_z verdicts");
  CHECK(coa_verify_batch_workspace_bytes(67) > 0, "coa_verify_batch_workspace_bytes");
  CHECK(coa_ed25519_verify_batch_device(0, NULL, NULL, NULL, 0, NULL, 1, NULL, NULL, 0, NULL) ==
            (gpu ? COA_EINVAL : COA_ENODEVICE),
        "verify_batch_device(null)");

  /* Digest */
  const uint8_t data[13] = {'H', 'e', 'l', 'l', 'o', ',', ' ', 'w', 'o', 'r', 'l', 'd', '!'};
  const uint64_t doff[2] = {0, 13};
  uint8_t out64[64], out32[32];
  CHECK(coa_sha512_many(data, doff, 1, out64) == dev_rc, "sha512_many");
  CHECK(coa_sha512_trunc32_many(data, doff, 1, out32) == dev_rc, "sha512_trunc32_many");
  CHECK(!gpu || memcmp(out32, msg, 32) == 0, "Digest(\"Hello, world!\")");
  CHECK(coa_sha512_many_device(0, NULL, NULL, 0, NULL, NULL) == dev_rc, "sha512_many_device(n=0)");

  /* committee cache + Certificate::verify */
  CHECK(coa_committee_register(pk, 1) == (gpu ? 1 : COA_ENODEVICE), "committee_register");
  uint32_t kf = 0;
  CHECK(coa_committee_key_flags(&kf, 1) == (gpu ? 1 : COA_ENODEVICE), "committee_key_flags");
  CHECK(coa_certificate_workspace_bytes(10, 670) > 0, "certificate_workspace_bytes");
  const uint64_t hoff[2] = {0, 13}, voff[2] = {0, 0}, rounds[1] = {1};
  uint8_t st = 9;
  CHECK(coa_certificate_verify_many(data, hoff, msg, pk, sig, rounds, NULL, NULL, voff, 1, 1, &st) == dev_rc,
        "certificate_verify_many");
  const int c1 = coa_certificate_verify(data, 13, msg, pk, sig, 1, NULL, NULL, 0, 1);
  CHECK(gpu ? c1 >= 0 : c1 == COA_ENODEVICE, "certificate_verify");
  CHECK(coa_certificate_verify_many_device(0, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, 0, 0, NULL,
                                           NULL, NULL) == dev_rc,
        "certificate_verify_many_device(n=0)");
  CHECK(coa_committee_register(NULL, 0) == (gpu ? 0 : COA_ENODEVICE), "committee_register(clear)");

  /* the engine's own CPU path: host-only, the same verdicts with or without
     a GPU (what the Rust policy answers with when every context failed) */
  CHECK(coa_cpu_ed25519_verify_strict(msg, 32, pk, sig) == COA_OK, "cpu verify_strict ok");
  CHECK(coa_cpu_ed25519_verify_strict(msg, 32, pk, bad) == COA_REJECT, "cpu verify_strict bad");
  uint8_t cv[2] = {9, 9};
  CHECK(coa_cpu_ed25519_verify_strict_many(msgs2, 32, pks2, sigs2, 2, cv, 2) == COA_OK && cv[0] == 0 && cv[1] == 1,
        "cpu verify_strict_many");
  CHECK(coa_cpu_ed25519_verify_batch(msg, pk, sig, 1, 5) == COA_OK, "cpu verify_batch ok");
  CHECK(coa_cpu_ed25519_verify_batch(msg, pk, bad, 1, 0) == COA_REJECT, "cpu verify_batch bad");
  uint8_t cg[2] = {9, 9};
  CHECK(coa_cpu_ed25519_verify_batch_groups_z(msgs2, pks2, sigs2, goff, 2, zs, cg, 0) == COA_OK && cg[0] == 0 &&
            cg[1] == 1,
        "cpu verify_batch_groups_z");
  uint8_t c64[64];
  CHECK(coa_cpu_sha512_many(data, doff, 1, c64, 1) == COA_OK && memcmp(c64, msg, 32) == 0, "cpu sha512_many");
  /* a certificate whose header hashes to `msg` ("Hello, world!"), signed
     header, no votes: only the header signature check can fail -- it is by
     the fixture's key over that very digest, so every bit is clear */
  uint8_t cst = 9;
  CHECK(coa_cpu_certificate_verify_many(data, hoff, msg, pk, sig, rounds, NULL, NULL, voff, 1, 3, &cst, 1) == COA_OK &&
            cst == 0,
        "cpu certificate_verify_many");
  CHECK(coa_cpu_certificate_verify_many_z(data, hoff, msg, pk, bad, rounds, NULL, NULL, voff, 1, NULL, &cst, 1) ==
                COA_OK &&
            cst == COA_CERT_BAD_HEADER_SIG,
        "cpu certificate_verify_many_z");
  CHECK(coa_cpu_ed25519_verify_strict_many(NULL, 32, NULL, NULL, 1, NULL, 1) == COA_EINVAL, "cpu (null)");

  /* wire decode: host-only, identical with or without a GPU */
  const uint8_t trunc[3] = {2, 0, 0};  /* a Certificate variant tag cut short */
  const uint64_t toff[2] = {0, 3};
  int32_t kind = 0;
  uint64_t hb = 0, nv = 0;
  CHECK(coa_wire_scan(trunc, toff, 1, &kind, &hb, &nv) == COA_OK && kind == COA_WIRE_ETRUNC, "wire_scan");
  {
    uint8_t hd[64], i32[32], o32[32], s64[64], vp[32], vs[64], au[32];
    uint64_t ho[2], r1[1], vo[2];
    uint32_t pc[1];
    CHECK(coa_wire_decode_certificates(trunc, toff, 0, hd, ho, i32, o32, s64, r1, vp, vs, vo, pc) == COA_OK,
          "wire_decode_certificates(n=0)");
    CHECK(coa_wire_decode_certificates(trunc, toff, 1, hd, ho, NULL, o32, s64, r1, vp, vs, vo, pc) == COA_EINVAL,
          "wire_decode_certificates(null ids)");
    CHECK(coa_wire_decode_votes(trunc, toff, 0, i32, r1, o32, au, s64) == COA_OK, "wire_decode_votes(n=0)");
    CHECK(coa_wire_decode_headers(trunc, toff, 0, hd, ho, i32, au, s64, r1, pc) == COA_OK,
          "wire_decode_headers(n=0)");
  }

  /* signing (input synthesis) */
  uint8_t seed[32], pk_out[32], sig_out[64];
  unhex(seed, "29b721769ce64e43d57133b074d839d531ed1f28510afb45ace10a1f4b794d6f", 32);
  CHECK(coa_ed25519_public_keys(seed, 1, pk_out) == dev_rc, "public_keys");
  CHECK(!gpu || memcmp(pk_out, pk, 32) == 0, "public_keys value");
  CHECK(coa_ed25519_sign_many(seed, msg, 32, 1, pk_out, sig_out) == dev_rc, "sign_many");
  CHECK(!gpu || memcmp(sig_out, sig, 64) == 0, "sign_many value (RFC 8032 deterministic)");
  CHECK(coa_ed25519_sign_many_device(0, NULL, NULL, 32, 0, NULL, NULL, NULL) == dev_rc, "sign_many_device(n=0)");

  /* aggregation queue */
  coa_queue* q = coa_queue_create(4, 100);
  CHECK(q != NULL, "queue_create");
  int seen = 99;
  CHECK(coa_queue_submit_verify(q, msg, pk, sig, cb, &seen) == COA_OK, "queue_submit_verify");
  CHECK(coa_queue_flush(q) == COA_OK, "queue_flush");
  CHECK(seen == dev_rc, "queue verify callback status");
  CHECK(coa_queue_submit_verify_many(q, msg, pk, sig, 1, cb, &seen) == COA_OK, "queue_submit_verify_many");
  CHECK(coa_queue_submit_verify_many(q, msg, pk, sig, 0, cb, &seen) == COA_EINVAL, "queue_submit_verify_many(n=0)");
  CHECK(coa_queue_flush(q) == COA_OK, "queue_flush many");
  CHECK(seen == dev_rc, "queue verify_many callback status");
  CHECK(coa_queue_submit_batch(q, msg, pk, sig, 1, cb, &seen) == COA_OK, "queue_submit_batch");
  CHECK(coa_queue_submit_certificate(q, data, 13, msg, pk, sig, 1, NULL, NULL, 0, cb, &seen) == COA_OK,
        "queue_submit_certificate");
  CHECK(coa_queue_submit_digest(q, data, 13, cb, &seen) == COA_OK, "queue_submit_digest");
  CHECK(coa_queue_submit_verify(q, msg, pk, sig, NULL, NULL) == COA_EINVAL, "queue_submit_verify(null cb)");
  CHECK(coa_queue_flush(q) == COA_OK, "queue_flush 2");
  CHECK(coa_queue_set_idle_launch(q, 1) == COA_OK && coa_queue_set_idle_launch(q, 0) == COA_OK &&
            coa_queue_set_idle_launch(q, 65) == COA_EINVAL && coa_queue_set_idle_launch(NULL, 1) == COA_EINVAL,
        "queue_set_idle_launch");
  uint64_t launches = 0, items = 0, groups = 0, digests = 0;
  CHECK(coa_queue_stats(q, &launches, &items, &groups) == COA_OK && items == 2 && groups == 2, "queue_stats");
  CHECK(coa_queue_digest_count(q, &digests) == COA_OK && digests == 1, "queue_digest_count");
  coa_queue_metrics_t qm;
  CHECK(coa_queue_metrics(q, &qm) == COA_OK && qm.requests == 5 && qm.signatures == 2 && qm.batches == 1 &&
            qm.certificates == 1 && qm.digests == 1 && qm.wait_us_max >= qm.wait_us_mean &&
            qm.retried_windows == qm.recovered_windows && qm.failed_windows == (gpu ? 0u : qm.windows),
        "queue_metrics");
  CHECK(coa_queue_metrics_reset(q) == COA_OK && coa_queue_metrics(q, &qm) == COA_OK && qm.requests == 0 &&
            qm.windows == 0 && qm.wait_us_p99 == 0.0 && qm.stage_us[COA_QSTAGE_CALLBACKS] == 0.0 &&
            (!gpu || qm.slots_verify > 0) && coa_queue_metrics_reset(NULL) == COA_EINVAL,
        "queue_metrics_reset");
  CHECK(coa_queue_destroy(q) == COA_OK, "queue_destroy");

  CHECK(coa_shutdown() == COA_OK, "coa_shutdown");
  if (failures) {
    fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  printf("abi harness ok (%s)\n", gpu ? "gpu" : "cpu");
  return 0;
}
