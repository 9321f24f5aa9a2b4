/* Second CPU reference for bench.py's cpu_baseline (SURVEY.md 8(d):
 * "libsodium crypto_sign_verify_detached where present").  Test / baseline
 * infrastructure only, like the rest of oracle/.
 *
 * libsodium is loaded with dlopen from the path the caller gives, so nothing
 * here needs its headers and the driver builds whether or not the image has
 * the library; a missing library is reported as -1 and the bench leaves the
 * second reference out.  Threads split [0, n) into contiguous ranges, the
 * same split coa_oracle_verify_strict_many uses, so the two baselines are
 * timed the same way. */
#include <dlfcn.h>
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>

typedef int (*verify_fn)(const unsigned char*, const unsigned char*, unsigned long long, const unsigned char*);

typedef struct {
  verify_fn f;
  const uint8_t *msgs, *pks, *sigs;
  size_t msg_len, lo, hi;
  uint8_t* out;
} sjob_t;

static void* sworker(void* p) {
  sjob_t* j = (sjob_t*)p;
  for (size_t i = j->lo; i < j->hi; i++)
    j->out[i] = j->f(j->sigs + 64 * i, j->msgs + j->msg_len * i, j->msg_len, j->pks + 32 * i) != 0;
  return NULL;
}

/* Returns 0, or -1 when the library or its symbols are absent.
 * version (may be null) receives sodium_version_string(). */
int coa_sodium_verify_many(const char* path, const uint8_t* msgs, size_t msg_len, const uint8_t* pks,
                           const uint8_t* sigs, size_t n, uint8_t* out, int nthreads, const char** version) {
  static void* h;
  static verify_fn f;
  static const char* ver;
  if (!h) {
    h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!h) return -1;
    int (*init)(void) = (int (*)(void))dlsym(h, "sodium_init");
    const char* (*vs)(void) = (const char* (*)(void))dlsym(h, "sodium_version_string");
    f = (verify_fn)dlsym(h, "crypto_sign_verify_detached");
    if (!init || !f || init() < 0) {
      f = NULL;
      return -1;
    }
    ver = vs ? vs() : "unknown";
  }
  if (!f) return -1;
  if (version) *version = ver;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  sjob_t jobs[256];
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = (sjob_t){f, msgs, pks, sigs, msg_len, n * t / nthreads, n * (t + 1) / nthreads, out};
    pthread_create(&th[t], NULL, sworker, &jobs[t]);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  return 0;
}
