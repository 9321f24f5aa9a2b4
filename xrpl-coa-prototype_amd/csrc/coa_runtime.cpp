// Host runtime behind include/coa_verify.h.
//
// * One context per GPU: a non-blocking HIP stream, the fixed-base B table
//   (built on the device by k_build_btable at coa_init) and growable device
//   buffers.  Each context has its own mutex; a call holds the mutexes of the
//   devices it enqueues on until their streams drain.
// * Host-pointer "many" calls shard items by contiguous index range over the
//   opened devices: no cross-GPU exchange, verdict bytes land
//   in place in the caller's output slice.
// * Device-pointer calls enqueue on the caller's stream and return.
// * No CPU fallback anywhere: without a usable GPU, calls fail with
//   COA_ENODEVICE.
#include "../../include/coa_verify.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <vector>

#include "coa_batch.h"
#include "coa_halved.h"
#include "coa_kernels.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                              \
  do {                                                                                             \
    hipError_t e_ = (expr);                                                                        \
    if (e_ != hipSuccess) return fail(COA_EHIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = std::max<size_t>(bytes + bytes / 4, 4096);
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

struct Dev {
  int id = 0;
  hipStream_t stream = nullptr;
  uint32_t* btab = nullptr;  // 128 x (j+1)B, radix-256 fixed-base table (12 KiB)
  uint32_t* comb = nullptr;  // 32 x 128 x (v+1)256^j B comb for k_verify_halved (384 KiB)
  DevBuf msgs, pks, sigs, kbuf, rec, verdicts, scratch, aux, rbuf, seeds, offs, data, out, idx, zs, terms, flags;
  std::mutex mu;
  std::vector<DevBuf*> all() {
    return {&msgs, &pks,  &sigs, &kbuf, &rec, &verdicts, &scratch, &aux,  &rbuf,
            &seeds, &offs, &data, &out,  &idx, &zs,       &terms,   &flags};
  }
};

// COA_VERIFY_IMPL=full selects the full-length k_verify_strict kernel (A/B
// and parity runs; read per call); the default is the halved-scalar path.
bool full_impl() {
  const char* impl = getenv("COA_VERIFY_IMPL");
  return impl && std::string(impl) == "full";
}
// COA_VERIFY_WAVES=3 selects the 168-VGPR instance of k_verify_halved.
int verify_waves() {
  const char* w = getenv("COA_VERIFY_WAVES");
  return (w && std::string(w) == "3") ? 3 : 2;
}

std::mutex g_init_mu;
std::vector<std::unique_ptr<Dev>> g_devs;
bool g_inited = false;

int init_locked(int n_gpus) {
  if (g_inited) return COA_OK;
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess || count <= 0)
    return fail(COA_ENODEVICE, "no HIP device available (this engine has no CPU fallback)");
  if (n_gpus <= 0 || n_gpus > count) n_gpus = count;
  for (int d = 0; d < n_gpus; d++) {
    auto dev = std::make_unique<Dev>();
    dev->id = d;
    HIP_TRY(hipSetDevice(d));
    HIP_TRY(hipStreamCreateWithFlags(&dev->stream, hipStreamNonBlocking));
    HIP_TRY(hipMalloc(&dev->btab, COA_BTAB_DWORDS * sizeof(uint32_t)));
    HIP_TRY(coa_launch_build_btable(dev->btab, dev->stream));
    HIP_TRY(hipMalloc(&dev->comb, COA_COMB_DWORDS * sizeof(uint32_t)));
    HIP_TRY(coa_launch_build_comb(dev->comb, dev->btab, dev->stream));
    HIP_TRY(hipStreamSynchronize(dev->stream));
    g_devs.push_back(std::move(dev));
  }
  g_inited = true;
  return COA_OK;
}

int ensure_init() {
  std::lock_guard<std::mutex> g(g_init_mu);
  return init_locked(0);
}

Dev* dev_by_id(int device) {
  for (auto& d : g_devs)
    if (d->id == device) return d.get();
  return nullptr;
}

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

uint32_t verify_lanes(size_t n) {
  const size_t lanes = align_up(std::max<size_t>(n, 1), COA_VERIFY_BLOCK);
  return (uint32_t)std::min<size_t>(lanes, COA_VERIFY_MAX_LANES);
}

struct Range {
  Dev* dev;
  size_t lo, hi;
};

// Contiguous index ranges [g*n/G, (g+1)*n/G) over the opened devices.
std::vector<Range> shard(size_t n) {
  std::vector<Range> r;
  const size_t G = g_devs.size();
  for (size_t g = 0; g < G; g++) {
    const size_t lo = n * g / G, hi = n * (g + 1) / G;
    if (hi > lo) r.push_back({g_devs[g].get(), lo, hi});
  }
  return r;
}

// Workspace layout for n items: k [n][32] | rec [n][128] | scratch [lanes][2 KiB]
struct Workspace {
  uint32_t* k;
  uint32_t* rec;
  uint32_t* scratch;
};
size_t ws_bytes(size_t n) {
  n = std::max<size_t>(n, 1);
  return align_up(n * 32, 256) + align_up(n * COA_HALVE_REC_BYTES, 256) +
         (size_t)verify_lanes(n) * COA_HALVED_SCRATCH_PER_LANE;
}
Workspace ws_carve(void* base, size_t n) {
  n = std::max<size_t>(n, 1);
  uint8_t* p = static_cast<uint8_t*>(base);
  Workspace w;
  w.k = reinterpret_cast<uint32_t*>(p);
  p += align_up(n * 32, 256);
  w.rec = reinterpret_cast<uint32_t*>(p);
  p += align_up(n * COA_HALVE_REC_BYTES, 256);
  w.scratch = reinterpret_cast<uint32_t*>(p);
  return w;
}

// Verify with k already in w.k: halved path (k_halve + k_verify_halved) or
// the full-length k_verify_strict.
int enqueue_verify_prehashed(Dev& d, const uint8_t* d_pks, const uint8_t* d_sigs, size_t n, uint8_t* d_verdicts,
                             const uint32_t* d_k, const Workspace& w, hipStream_t s) {
  const uint32_t lanes = verify_lanes(n);
  if (full_impl()) {
    HIP_TRY(coa_launch_verify_strict(d_pks, d_sigs, d_k, (uint32_t)n, d_verdicts, w.scratch, lanes, d.btab, s));
    return COA_OK;
  }
  HIP_TRY(coa_launch_halve(d_k, d_sigs, (uint32_t)n, w.rec, s));
  HIP_TRY(coa_launch_verify_halved(d_pks, d_sigs, w.rec, (uint32_t)n, d_verdicts, w.scratch, lanes, d.comb,
                                   verify_waves(), s));
  return COA_OK;
}

// Enqueue k = H(R||A||M) then the verification for device-resident inputs.
int enqueue_verify(Dev& d, const uint8_t* d_msgs, size_t msg_len, const uint8_t* d_pks, const uint8_t* d_sigs,
                   size_t n, uint8_t* d_verdicts, const Workspace& w, hipStream_t s) {
  HIP_TRY(coa_launch_hram(d_msgs, (uint32_t)msg_len, msg_len, nullptr, d_pks, d_sigs, (uint32_t)n, w.k, s));
  return enqueue_verify_prehashed(d, d_pks, d_sigs, n, d_verdicts, w.k, w, s);
}

int check_n(size_t n) {
  if (n > 0xffffffffull / 2) return fail(COA_EINVAL, "n too large for one call");
  return COA_OK;
}

// Run `body` for every shard with the device lock held, then drain every
// used stream.  body(Dev&, lo, hi) enqueues work and returns COA_OK or an error.
template <class F>
int for_shards(size_t n, F body) {
  std::vector<Range> rs = shard(n);
  std::vector<std::unique_lock<std::mutex>> locks;
  int rc = COA_OK;
  for (auto& r : rs) {
    locks.emplace_back(r.dev->mu);
    if (hipSetDevice(r.dev->id) != hipSuccess) {
      rc = fail(COA_EHIP, "hipSetDevice failed");
      break;
    }
    rc = body(*r.dev, r.lo, r.hi);
    if (rc != COA_OK) break;
  }
  for (auto& r : rs) {
    (void)hipSetDevice(r.dev->id);
    hipError_t e = hipStreamSynchronize(r.dev->stream);
    if (e != hipSuccess && rc == COA_OK) rc = fail(COA_EHIP, std::string("stream sync: ") + hipGetErrorString(e));
  }
  return rc;
}

uint64_t os_entropy_seed() {
  std::random_device rd;
  uint64_t s = 0;
  while (s == 0) s = ((uint64_t)rd() << 32) ^ rd();
  return s;
}

int batch_groups_impl(const uint8_t* msgs, const uint8_t* pks, const uint8_t* sigs, const uint64_t* group_offsets,
                      size_t n_groups, const uint8_t* zs_in, uint64_t seed, uint8_t* verdicts_out) {
  if (n_groups == 0) return COA_OK;
  if (!msgs || !group_offsets || !verdicts_out) return fail(COA_EINVAL, "null argument");
  if (group_offsets[0] != 0) return fail(COA_EINVAL, "group_offsets[0] must be 0");
  for (size_t g = 0; g < n_groups; g++)
    if (group_offsets[g + 1] < group_offsets[g]) return fail(COA_EINVAL, "group_offsets not monotone");
  const size_t total = group_offsets[n_groups];
  if (total && (!pks || !sigs)) return fail(COA_EINVAL, "null pks/sigs");
  if (check_n(total) != COA_OK) return COA_EINVAL;
  const uint64_t eff_seed = zs_in ? 0 : (seed ? seed : os_entropy_seed());
  // shard by group index
  return for_shards(n_groups, [&](Dev& d, size_t glo, size_t ghi) -> int {
    const size_t vlo = group_offsets[glo], vhi = group_offsets[ghi];
    const size_t nv = vhi - vlo, ng = ghi - glo;
    std::vector<uint64_t> offs(ng + 1);
    std::vector<uint32_t> group_of(std::max<size_t>(nv, 1));
    for (size_t g = 0; g <= ng; g++) offs[g] = group_offsets[glo + g] - vlo;
    for (size_t g = 0; g < ng; g++)
      for (uint64_t i = offs[g]; i < offs[g + 1]; i++) group_of[i] = (uint32_t)(glo + g);
    const uint32_t lanes = verify_lanes(nv);
    hipStream_t s = d.stream;
    HIP_TRY(d.msgs.ensure(ng * 32));
    HIP_TRY(d.pks.ensure(nv * 32 + 32));
    HIP_TRY(d.sigs.ensure(nv * 64 + 64));
    HIP_TRY(d.kbuf.ensure(nv * 32 + 32));
    HIP_TRY(d.zs.ensure(nv * 16 + 16));
    HIP_TRY(d.idx.ensure(group_of.size() * 4));
    HIP_TRY(d.offs.ensure((ng + 1) * 8));
    HIP_TRY(d.terms.ensure(nv * 128 + 128));
    HIP_TRY(d.flags.ensure(nv + 16));
    HIP_TRY(d.scratch.ensure((size_t)lanes * COA_BATCH_SCRATCH_PER_LANE));
    HIP_TRY(d.verdicts.ensure(ng + 16));
    HIP_TRY(hipMemcpyAsync(d.msgs.p, msgs + glo * 32, ng * 32, hipMemcpyHostToDevice, s));
    if (nv) {
      HIP_TRY(hipMemcpyAsync(d.pks.p, pks + vlo * 32, nv * 32, hipMemcpyHostToDevice, s));
      HIP_TRY(hipMemcpyAsync(d.sigs.p, sigs + vlo * 64, nv * 64, hipMemcpyHostToDevice, s));
    }
    // group ids are relative to this shard's message slice
    for (auto& gid : group_of) gid -= (uint32_t)glo;
    HIP_TRY(hipMemcpyAsync(d.idx.p, group_of.data(), group_of.size() * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d.offs.p, offs.data(), (ng + 1) * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(coa_launch_hram(d.msgs.as<uint8_t>(), 32, 32, d.idx.as<uint32_t>(), d.pks.as<uint8_t>(),
                            d.sigs.as<uint8_t>(), (uint32_t)nv, d.kbuf.as<uint32_t>(), s));
    if (zs_in) {
      if (nv) HIP_TRY(hipMemcpyAsync(d.zs.p, zs_in + vlo * 16, nv * 16, hipMemcpyHostToDevice, s));
    } else {
      // z derivation binds the global group index: restore it for the hash
      std::vector<uint32_t> gabs(group_of.size());
      for (size_t i = 0; i < group_of.size(); i++) gabs[i] = group_of[i] + (uint32_t)glo;
      HIP_TRY(hipMemcpyAsync(d.idx.p, gabs.data(), gabs.size() * 4, hipMemcpyHostToDevice, s));
      HIP_TRY(coa_launch_batch_z(d.kbuf.as<uint32_t>(), d.sigs.as<uint8_t>(), d.idx.as<uint32_t>(), (uint32_t)nv,
                                 eff_seed, d.zs.as<uint32_t>(), s));
      HIP_TRY(hipStreamSynchronize(s));  // gabs lifetime
    }
    HIP_TRY(coa_launch_batch_terms(d.pks.as<uint8_t>(), d.sigs.as<uint8_t>(), d.kbuf.as<uint32_t>(),
                                   d.zs.as<uint32_t>(), (uint32_t)nv, d.terms.as<uint32_t>(), d.flags.as<uint8_t>(),
                                   d.scratch.as<uint32_t>(), lanes, d.btab, s));
    HIP_TRY(coa_launch_batch_reduce(d.offs.as<uint64_t>(), (uint32_t)ng, d.terms.as<uint32_t>(),
                                    d.flags.as<uint8_t>(), d.verdicts.as<uint8_t>(), s));
    HIP_TRY(hipMemcpyAsync(verdicts_out + glo, d.verdicts.p, ng, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));  // offs / group_of host vectors die here
    return COA_OK;
  });
}

int sign_enqueue(Dev& d, const uint8_t* d_seeds, const uint8_t* d_msgs, size_t msg_len, size_t n, uint8_t* d_pks,
                 uint8_t* d_sigs, hipStream_t s) {
  HIP_TRY(d.aux.ensure(n * 64 + 64));
  HIP_TRY(d.rbuf.ensure(n * 32 + 32));
  HIP_TRY(d.kbuf.ensure(n * 32 + 32));
  HIP_TRY(coa_launch_keygen(d_seeds, (uint32_t)n, d_pks, d.aux.as<uint32_t>(), d.btab, s));
  HIP_TRY(coa_launch_sign_r(d.aux.as<uint32_t>(), d_msgs, (uint32_t)msg_len, (uint32_t)n, d_sigs,
                            d.rbuf.as<uint32_t>(), d.btab, s));
  HIP_TRY(coa_launch_hram(d_msgs, (uint32_t)msg_len, msg_len, nullptr, d_pks, d_sigs, (uint32_t)n,
                          d.kbuf.as<uint32_t>(), s));
  HIP_TRY(coa_launch_sign_s(d.aux.as<uint32_t>(), d.rbuf.as<uint32_t>(), d.kbuf.as<uint32_t>(), (uint32_t)n, d_sigs,
                            s));
  return COA_OK;
}

}  // namespace

extern "C" {

const char* coa_last_error(void) { return g_err.c_str(); }
const char* coa_version(void) { return "coa_verify 0.1.0 gfx950"; }

int coa_init(int n_gpus) {
  std::lock_guard<std::mutex> g(g_init_mu);
  return init_locked(n_gpus);
}

int coa_shutdown(void) {
  std::lock_guard<std::mutex> g(g_init_mu);
  for (auto& d : g_devs) {
    std::lock_guard<std::mutex> l(d->mu);
    (void)hipSetDevice(d->id);
    (void)hipStreamSynchronize(d->stream);
    for (DevBuf* b : d->all()) b->release();
    if (d->btab) (void)hipFree(d->btab);
    if (d->comb) (void)hipFree(d->comb);
    (void)hipStreamDestroy(d->stream);
  }
  g_devs.clear();
  g_inited = false;
  return COA_OK;
}

int coa_device_count(void) {
  const int r = ensure_init();
  if (r != COA_OK) return r;
  return (int)g_devs.size();
}

size_t coa_verify_workspace_bytes(size_t n) { return ws_bytes(n); }

int coa_ed25519_verify_strict_many(const uint8_t* msgs, size_t msg_len, const uint8_t* pks, const uint8_t* sigs,
                                   size_t n, uint8_t* verdicts_out) {
  int rc = ensure_init();
  if (rc != COA_OK) return rc;
  if (n == 0) return COA_OK;
  if ((!msgs && msg_len) || !pks || !sigs || !verdicts_out) return fail(COA_EINVAL, "null argument");
  if (check_n(n) != COA_OK) return COA_EINVAL;
  return for_shards(n, [&](Dev& d, size_t lo, size_t hi) -> int {
    const size_t cnt = hi - lo;
    hipStream_t s = d.stream;
    HIP_TRY(d.msgs.ensure(cnt * msg_len + 4));
    HIP_TRY(d.pks.ensure(cnt * 32));
    HIP_TRY(d.sigs.ensure(cnt * 64));
    HIP_TRY(d.scratch.ensure(ws_bytes(cnt)));
    HIP_TRY(d.verdicts.ensure(cnt));
    if (msg_len) HIP_TRY(hipMemcpyAsync(d.msgs.p, msgs + lo * msg_len, cnt * msg_len, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d.pks.p, pks + lo * 32, cnt * 32, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d.sigs.p, sigs + lo * 64, cnt * 64, hipMemcpyHostToDevice, s));
    int r = enqueue_verify(d, d.msgs.as<uint8_t>(), msg_len, d.pks.as<uint8_t>(), d.sigs.as<uint8_t>(), cnt,
                           d.verdicts.as<uint8_t>(), ws_carve(d.scratch.p, cnt), s);
    if (r != COA_OK) return r;
    HIP_TRY(hipMemcpyAsync(verdicts_out + lo, d.verdicts.p, cnt, hipMemcpyDeviceToHost, s));
    return COA_OK;
  });
}

int coa_ed25519_verify_strict(const uint8_t msg[32], const uint8_t pk[32], const uint8_t sig[64]) {
  uint8_t v = 1;
  const int rc = coa_ed25519_verify_strict_many(msg, 32, pk, sig, 1, &v);
  if (rc != COA_OK) return rc;
  return v ? COA_REJECT : COA_OK;
}

int coa_ed25519_verify_strict_many_device(int device, const uint8_t* d_msgs, size_t msg_len, const uint8_t* d_pks,
                                          const uint8_t* d_sigs, size_t n, uint8_t* d_verdicts, void* workspace,
                                          void* stream) {
  int rc = ensure_init();
  if (rc != COA_OK) return rc;
  if (n == 0) return COA_OK;
  if ((!d_msgs && msg_len) || !d_pks || !d_sigs || !d_verdicts) return fail(COA_EINVAL, "null argument");
  if (check_n(n) != COA_OK) return COA_EINVAL;
  Dev* d = dev_by_id(device);
  if (!d) return fail(COA_EINVAL, "device not opened by coa_init");
  HIP_TRY(hipSetDevice(device));
  hipStream_t s = stream ? (hipStream_t)stream : d->stream;
  if (workspace) return enqueue_verify(*d, d_msgs, msg_len, d_pks, d_sigs, n, d_verdicts, ws_carve(workspace, n), s);
  std::lock_guard<std::mutex> l(d->mu);
  HIP_TRY(d->scratch.ensure(ws_bytes(n)));
  rc = enqueue_verify(*d, d_msgs, msg_len, d_pks, d_sigs, n, d_verdicts, ws_carve(d->scratch.p, n), s);
  if (rc != COA_OK) return rc;
  HIP_TRY(hipStreamSynchronize(s));  // engine-owned workspace: drain before release
  return COA_OK;
}

int coa_ed25519_challenge_many_device(int device, const uint8_t* d_msgs, size_t msg_len, const uint8_t* d_pks,
                                      const uint8_t* d_sigs, size_t n, uint8_t* d_k_out, void* stream) {
  int rc = ensure_init();
  if (rc != COA_OK) return rc;
  if (n == 0) return COA_OK;
  if ((!d_msgs && msg_len) || !d_pks || !d_sigs || !d_k_out) return fail(COA_EINVAL, "null argument");
  if (check_n(n) != COA_OK) return COA_EINVAL;
  Dev* d = dev_by_id(device);
  if (!d) return fail(COA_EINVAL, "device not opened by coa_init");
  HIP_TRY(hipSetDevice(device));
  hipStream_t s = stream ? (hipStream_t)stream : d->stream;
  HIP_TRY(coa_launch_hram(d_msgs, (uint32_t)msg_len, msg_len, nullptr, d_pks, d_sigs, (uint32_t)n,
                          reinterpret_cast<uint32_t*>(d_k_out), s));
  return COA_OK;
}

int coa_ed25519_verify_prehashed_many_device(int device, const uint8_t* d_k, const uint8_t* d_pks,
                                             const uint8_t* d_sigs, size_t n, uint8_t* d_verdicts, void* workspace,
                                             void* stream) {
  int rc = ensure_init();
  if (rc != COA_OK) return rc;
  if (n == 0) return COA_OK;
  if (!d_k || !d_pks || !d_sigs || !d_verdicts) return fail(COA_EINVAL, "null argument");
  if (check_n(n) != COA_OK) return COA_EINVAL;
  Dev* d = dev_by_id(device);
  if (!d) return fail(COA_EINVAL, "device not opened by coa_init");
  HIP_TRY(hipSetDevice(device));
  hipStream_t s = stream ? (hipStream_t)stream : d->stream;
  const uint32_t* k = reinterpret_cast<const uint32_t*>(d_k);
  if (workspace) return enqueue_verify_prehashed(*d, d_pks, d_sigs, n, d_verdicts, k, ws_carve(workspace, n), s);
  std::lock_guard<std::mutex> l(d->mu);
  HIP_TRY(d->scratch.ensure(ws_bytes(n)));
  rc = enqueue_verify_prehashed(*d, d_pks, d_sigs, n, d_verdicts, k, ws_carve(d->scratch.p, n), s);
  if (rc != COA_OK) return rc;
  HIP_TRY(hipStreamSynchronize(s));
  return COA_OK;
}

int coa_ed25519_verify_batch_groups(const uint8_t* msgs, const uint8_t* pks, const uint8_t* sigs,
                                    const uint64_t* group_offsets, size_t n_groups, uint8_t* group_verdicts_out,
                                    uint64_t rng_seed) {
  int rc = ensure_init();
  if (rc != COA_OK) return rc;
  return batch_groups_impl(msgs, pks, sigs, group_offsets, n_groups, nullptr, rng_seed, group_verdicts_out);
}

int coa_ed25519_verify_batch_groups_z(const uint8_t* msgs, const uint8_t* pks, const uint8_t* sigs,
                                      const uint64_t* group_offsets, size_t n_groups, const uint8_t* zs,
                                      uint8_t* group_verdicts_out) {
  int rc = ensure_init();
  if (rc != COA_OK) return rc;
  if (!zs && n_groups && group_offsets && group_offsets[n_groups]) return fail(COA_EINVAL, "null zs");
  static const uint8_t zero16[16] = {0};
  return batch_groups_impl(msgs, pks, sigs, group_offsets, n_groups, zs ? zs : zero16, 0, group_verdicts_out);
}

int coa_ed25519_verify_batch(const uint8_t msg[32], const uint8_t* pks, const uint8_t* sigs, size_t n,
                             uint64_t rng_seed) {
  const uint64_t offs[2] = {0, (uint64_t)n};
  uint8_t v = 1;
  const int rc = coa_ed25519_verify_batch_groups(msg, pks, sigs, offs, 1, &v, rng_seed);
  if (rc != COA_OK) return rc;
  return v ? COA_REJECT : COA_OK;
}

int coa_sha512_many(const uint8_t* data, const uint64_t* offsets, size_t n, uint8_t* out64) {
  int rc = ensure_init();
  if (rc != COA_OK) return rc;
  if (n == 0) return COA_OK;
  if (!offsets || !out64) return fail(COA_EINVAL, "null argument");
  for (size_t i = 0; i < n; i++)
    if (offsets[i + 1] < offsets[i]) return fail(COA_EINVAL, "offsets not monotone");
  if (offsets[n] > offsets[0] && !data) return fail(COA_EINVAL, "null data");
  if (check_n(n) != COA_OK) return COA_EINVAL;
  return for_shards(n, [&](Dev& d, size_t lo, size_t hi) -> int {
    const size_t cnt = hi - lo;
    const uint64_t base = offsets[lo], bytes = offsets[hi] - base;
    std::vector<uint64_t> rel(cnt + 1);
    for (size_t i = 0; i <= cnt; i++) rel[i] = offsets[lo + i] - base;
    hipStream_t s = d.stream;
    HIP_TRY(d.data.ensure(bytes + 16));
    HIP_TRY(d.offs.ensure((cnt + 1) * 8));
    HIP_TRY(d.out.ensure(cnt * 64));
    if (bytes) HIP_TRY(hipMemcpyAsync(d.data.p, data + base, bytes, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d.offs.p, rel.data(), (cnt + 1) * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(coa_launch_sha512_many(d.data.as<uint8_t>(), d.offs.as<uint64_t>(), (uint32_t)cnt,
                                   d.out.as<uint32_t>(), s));
    HIP_TRY(hipMemcpyAsync(out64 + lo * 64, d.out.p, cnt * 64, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));  // rel dies here
    return COA_OK;
  });
}

int coa_sha512_trunc32_many(const uint8_t* data, const uint64_t* offsets, size_t n, uint8_t* out32) {
  if (n == 0) return ensure_init();
  if (!out32) return fail(COA_EINVAL, "null argument");
  std::vector<uint8_t> full(n * 64);
  const int rc = coa_sha512_many(data, offsets, n, full.data());
  if (rc != COA_OK) return rc;
  for (size_t i = 0; i < n; i++) std::memcpy(out32 + i * 32, full.data() + i * 64, 32);
  return COA_OK;
}

int coa_sha512_many_device(int device, const uint8_t* d_data, const uint64_t* d_offsets, size_t n, uint8_t* d_out64,
                           void* stream) {
  int rc = ensure_init();
  if (rc != COA_OK) return rc;
  if (n == 0) return COA_OK;
  if (!d_data || !d_offsets || !d_out64) return fail(COA_EINVAL, "null argument");
  if (check_n(n) != COA_OK) return COA_EINVAL;
  Dev* d = dev_by_id(device);
  if (!d) return fail(COA_EINVAL, "device not opened by coa_init");
  HIP_TRY(hipSetDevice(device));
  hipStream_t s = stream ? (hipStream_t)stream : d->stream;
  HIP_TRY(coa_launch_sha512_many(d_data, d_offsets, (uint32_t)n, reinterpret_cast<uint32_t*>(d_out64), s));
  return COA_OK;
}

int coa_ed25519_sign_many(const uint8_t* seeds, const uint8_t* msgs, size_t msg_len, size_t n, uint8_t* pks_out,
                          uint8_t* sigs_out) {
  int rc = ensure_init();
  if (rc != COA_OK) return rc;
  if (n == 0) return COA_OK;
  if (!seeds || (!msgs && msg_len) || !pks_out || !sigs_out) return fail(COA_EINVAL, "null argument");
  if (check_n(n) != COA_OK) return COA_EINVAL;
  return for_shards(n, [&](Dev& d, size_t lo, size_t hi) -> int {
    const size_t cnt = hi - lo;
    hipStream_t s = d.stream;
    HIP_TRY(d.seeds.ensure(cnt * 32));
    HIP_TRY(d.msgs.ensure(cnt * msg_len + 4));
    HIP_TRY(d.pks.ensure(cnt * 32));
    HIP_TRY(d.sigs.ensure(cnt * 64));
    HIP_TRY(hipMemcpyAsync(d.seeds.p, seeds + lo * 32, cnt * 32, hipMemcpyHostToDevice, s));
    if (msg_len) HIP_TRY(hipMemcpyAsync(d.msgs.p, msgs + lo * msg_len, cnt * msg_len, hipMemcpyHostToDevice, s));
    int r = sign_enqueue(d, d.seeds.as<uint8_t>(), d.msgs.as<uint8_t>(), msg_len, cnt, d.pks.as<uint8_t>(),
                         d.sigs.as<uint8_t>(), s);
    if (r != COA_OK) return r;
    HIP_TRY(hipMemcpyAsync(pks_out + lo * 32, d.pks.p, cnt * 32, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(sigs_out + lo * 64, d.sigs.p, cnt * 64, hipMemcpyDeviceToHost, s));
    return COA_OK;
  });
}

int coa_ed25519_public_keys(const uint8_t* seeds, size_t n, uint8_t* pks_out) {
  int rc = ensure_init();
  if (rc != COA_OK) return rc;
  if (n == 0) return COA_OK;
  if (!seeds || !pks_out) return fail(COA_EINVAL, "null argument");
  if (check_n(n) != COA_OK) return COA_EINVAL;
  return for_shards(n, [&](Dev& d, size_t lo, size_t hi) -> int {
    const size_t cnt = hi - lo;
    hipStream_t s = d.stream;
    HIP_TRY(d.seeds.ensure(cnt * 32));
    HIP_TRY(d.pks.ensure(cnt * 32));
    HIP_TRY(d.aux.ensure(cnt * 64));
    HIP_TRY(hipMemcpyAsync(d.seeds.p, seeds + lo * 32, cnt * 32, hipMemcpyHostToDevice, s));
    HIP_TRY(coa_launch_keygen(d.seeds.as<uint8_t>(), (uint32_t)cnt, d.pks.as<uint8_t>(), d.aux.as<uint32_t>(),
                              d.btab, s));
    HIP_TRY(hipMemcpyAsync(pks_out + lo * 32, d.pks.p, cnt * 32, hipMemcpyDeviceToHost, s));
    return COA_OK;
  });
}

int coa_ed25519_sign_many_device(int device, const uint8_t* d_seeds, const uint8_t* d_msgs, size_t msg_len, size_t n,
                                 uint8_t* d_pks_out, uint8_t* d_sigs_out, void* stream) {
  int rc = ensure_init();
  if (rc != COA_OK) return rc;
  if (n == 0) return COA_OK;
  if (!d_seeds || (!d_msgs && msg_len) || !d_pks_out || !d_sigs_out) return fail(COA_EINVAL, "null argument");
  if (check_n(n) != COA_OK) return COA_EINVAL;
  Dev* d = dev_by_id(device);
  if (!d) return fail(COA_EINVAL, "device not opened by coa_init");
  HIP_TRY(hipSetDevice(device));
  std::lock_guard<std::mutex> l(d->mu);
  hipStream_t s = stream ? (hipStream_t)stream : d->stream;
  rc = sign_enqueue(*d, d_seeds, d_msgs, msg_len, n, d_pks_out, d_sigs_out, s);
  if (rc != COA_OK) return rc;
  HIP_TRY(hipStreamSynchronize(s));
  return COA_OK;
}

}  // extern "C"
