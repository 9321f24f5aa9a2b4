// Aggregation queue: the pre-verification stage between
// PrimaryReceiverHandler::dispatch (primary/src/primary.rs:223-244) and
// Core (primary/src/core.rs:349-389).  Core verifies one message at a time;
// this stage collects pending header/vote signatures and certificate vote
// batches from any number of producer threads and launches them as a few
// large GPU calls.  Modelled on the reference's SignatureService
// (crypto/src/lib.rs:222-250): a request channel in, a per-request reply
// (here a C callback, which the Rust side maps onto a oneshot channel).
//
// Four request kinds, each coalesced into one engine call per launch:
//   verify       header / vote signatures -> coa_ed25519_verify_strict_many
//   batch        bare vote batches        -> coa_ed25519_verify_batch_groups
//   certificate  whole Certificate::verify crypto (f3)
//                                         -> coa_certificate_verify_many
//   digest       worker batch digests (worker/src/processor.rs:38; the
//                Processor loop hashes one batch at a time)
//                                         -> coa_sha512_trunc32_many
// A launch happens when `max_batch` items are pending (a signature, a vote
// or a digest each count one), when the oldest request is `max_delay_us`
// old, or on coa_queue_flush.  Inputs are copied at submission; callbacks
// run on the queue's worker thread.
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/coa_verify.h"

namespace {

using clock_t_ = std::chrono::steady_clock;

struct Single {
  uint8_t msg[32], pk[32], sig[64];
  coa_verdict_cb cb;
  void* user;
};

struct Group {
  uint8_t msg[32];
  std::vector<uint8_t> pks, sigs;
  coa_verdict_cb cb;
  void* user;
};

struct Cert {
  std::vector<uint8_t> header, pks, sigs;
  uint8_t id[32], origin[32], hsig[64];
  uint64_t round;
  coa_verdict_cb cb;
  void* user;
};

struct Dig {
  std::vector<uint8_t> data;
  coa_verdict_cb cb;
  void* user;
};

}  // namespace

struct coa_queue {
  size_t max_batch;
  std::chrono::microseconds max_delay;
  std::mutex mu;
  std::condition_variable cv, idle_cv;
  std::vector<Single> singles;
  std::vector<Group> groups;
  std::vector<Cert> certs;
  std::vector<Dig> digs;
  size_t pending_sigs = 0;
  clock_t_::time_point oldest;
  bool flush = false, stop = false, busy = false;
  uint64_t launches = 0, items = 0, ngroups = 0, ndigests = 0;
  std::thread worker;

  void run() {
    std::unique_lock<std::mutex> l(mu);
    for (;;) {
      cv.wait(l, [&] { return stop || pending_sigs > 0; });
      if (pending_sigs == 0) return;  // stop with nothing pending
      // batch is open: launch when full, at the deadline, on flush or stop
      while (!stop && !flush && pending_sigs < max_batch) {
        if (cv.wait_until(l, oldest + max_delay) == std::cv_status::timeout) break;
      }
      std::vector<Single> s;
      std::vector<Group> g;
      std::vector<Cert> c;
      std::vector<Dig> d;
      s.swap(singles);
      g.swap(groups);
      c.swap(certs);
      d.swap(digs);
      pending_sigs = 0;
      busy = true;
      l.unlock();
      launch(s, g);
      launch_certs(c);
      launch_digests(d);
      l.lock();
      busy = false;
      launches++;
      items += s.size();
      ngroups += g.size() + c.size();
      ndigests += d.size();
      if (pending_sigs == 0) {
        flush = false;
        idle_cv.notify_all();
      }
    }
  }

  static void launch(std::vector<Single>& s, std::vector<Group>& g) {
    if (!s.empty()) {
      const size_t n = s.size();
      std::vector<uint8_t> msgs(n * 32), pks(n * 32), sigs(n * 64), out(n, 1);
      for (size_t i = 0; i < n; i++) {
        std::memcpy(&msgs[i * 32], s[i].msg, 32);
        std::memcpy(&pks[i * 32], s[i].pk, 32);
        std::memcpy(&sigs[i * 64], s[i].sig, 64);
      }
      const int rc = coa_ed25519_verify_strict_many(msgs.data(), 32, pks.data(), sigs.data(), n, out.data());
      for (size_t i = 0; i < n; i++) s[i].cb(s[i].user, rc, &out[i], 1);
    }
    if (!g.empty()) {
      const size_t ng = g.size();
      std::vector<uint8_t> msgs(ng * 32), pks, sigs, out(ng, 1);
      std::vector<uint64_t> offs(ng + 1, 0);
      for (size_t i = 0; i < ng; i++) {
        std::memcpy(&msgs[i * 32], g[i].msg, 32);
        pks.insert(pks.end(), g[i].pks.begin(), g[i].pks.end());
        sigs.insert(sigs.end(), g[i].sigs.begin(), g[i].sigs.end());
        offs[i + 1] = offs[i] + g[i].pks.size() / 32;
      }
      const int rc = coa_ed25519_verify_batch_groups(msgs.data(), pks.data(), sigs.data(), offs.data(), ng,
                                                     out.data(), 0);
      for (size_t i = 0; i < ng; i++) g[i].cb(g[i].user, rc, &out[i], 1);
    }
  }

  static void launch_certs(std::vector<Cert>& c) {
    if (c.empty()) return;
    const size_t n = c.size();
    std::vector<uint8_t> hdata, ids(n * 32), origins(n * 32), hsigs(n * 64), pks, sigs, out(n, 7);
    std::vector<uint64_t> hoff(n + 1, 0), voff(n + 1, 0), rounds(n);
    for (size_t i = 0; i < n; i++) {
      hdata.insert(hdata.end(), c[i].header.begin(), c[i].header.end());
      hoff[i + 1] = hdata.size();
      std::memcpy(&ids[i * 32], c[i].id, 32);
      std::memcpy(&origins[i * 32], c[i].origin, 32);
      std::memcpy(&hsigs[i * 64], c[i].hsig, 64);
      rounds[i] = c[i].round;
      pks.insert(pks.end(), c[i].pks.begin(), c[i].pks.end());
      sigs.insert(sigs.end(), c[i].sigs.begin(), c[i].sigs.end());
      voff[i + 1] = voff[i] + c[i].pks.size() / 32;
    }
    const int rc = coa_certificate_verify_many(hdata.data(), hoff.data(), ids.data(), origins.data(), hsigs.data(),
                                               rounds.data(), pks.data(), sigs.data(), voff.data(), n, 0,
                                               out.data());
    for (size_t i = 0; i < n; i++) c[i].cb(c[i].user, rc, &out[i], 1);
  }

  static void launch_digests(std::vector<Dig>& d) {
    if (d.empty()) return;
    const size_t n = d.size();
    std::vector<uint8_t> data, out(n * 32, 0);
    std::vector<uint64_t> offs(n + 1, 0);
    for (size_t i = 0; i < n; i++) {
      data.insert(data.end(), d[i].data.begin(), d[i].data.end());
      offs[i + 1] = data.size();
    }
    const int rc = coa_sha512_trunc32_many(data.data(), offs.data(), n, out.data());
    for (size_t i = 0; i < n; i++) d[i].cb(d[i].user, rc, &out[i * 32], 32);
  }

  void note_arrival(size_t sigs) {
    const bool first = pending_sigs == 0;
    if (first) oldest = clock_t_::now();
    pending_sigs += sigs;
    if (first || pending_sigs >= max_batch) cv.notify_one();  // arm the deadline / launch a full batch
  }
};

extern "C" {

coa_queue* coa_queue_create(size_t max_batch, uint32_t max_delay_us) {
  coa_queue* q = new coa_queue();
  q->max_batch = max_batch ? max_batch : 65536;
  q->max_delay = std::chrono::microseconds(max_delay_us);
  q->worker = std::thread([q] { q->run(); });
  return q;
}

int coa_queue_submit_verify(coa_queue* q, const uint8_t msg[32], const uint8_t pk[32], const uint8_t sig[64],
                            coa_verdict_cb cb, void* user) {
  if (!q || !msg || !pk || !sig || !cb) return COA_EINVAL;
  Single s;
  std::memcpy(s.msg, msg, 32);
  std::memcpy(s.pk, pk, 32);
  std::memcpy(s.sig, sig, 64);
  s.cb = cb;
  s.user = user;
  std::lock_guard<std::mutex> l(q->mu);
  if (q->stop) return COA_EINVAL;
  q->singles.push_back(s);
  q->note_arrival(1);
  return COA_OK;
}

int coa_queue_submit_batch(coa_queue* q, const uint8_t msg[32], const uint8_t* pks, const uint8_t* sigs, size_t n,
                           coa_verdict_cb cb, void* user) {
  if (!q || !msg || (n && (!pks || !sigs)) || !cb) return COA_EINVAL;
  Group g;
  std::memcpy(g.msg, msg, 32);
  g.pks.assign(pks, pks + n * 32);
  g.sigs.assign(sigs, sigs + n * 64);
  g.cb = cb;
  g.user = user;
  std::lock_guard<std::mutex> l(q->mu);
  if (q->stop) return COA_EINVAL;
  q->groups.push_back(std::move(g));
  q->note_arrival(n ? n : 1);
  return COA_OK;
}

int coa_queue_submit_certificate(coa_queue* q, const uint8_t* header_data, size_t header_len, const uint8_t id[32],
                                 const uint8_t origin[32], const uint8_t header_sig[64], uint64_t round,
                                 const uint8_t* vote_pks, const uint8_t* vote_sigs, size_t n_votes, coa_verdict_cb cb,
                                 void* user) {
  if (!q || (header_len && !header_data) || !id || !origin || !header_sig || (n_votes && (!vote_pks || !vote_sigs)) ||
      !cb)
    return COA_EINVAL;
  Cert c;
  c.header.assign(header_data, header_data + header_len);
  std::memcpy(c.id, id, 32);
  std::memcpy(c.origin, origin, 32);
  std::memcpy(c.hsig, header_sig, 64);
  c.round = round;
  c.pks.assign(vote_pks, vote_pks + n_votes * 32);
  c.sigs.assign(vote_sigs, vote_sigs + n_votes * 64);
  c.cb = cb;
  c.user = user;
  std::lock_guard<std::mutex> l(q->mu);
  if (q->stop) return COA_EINVAL;
  q->certs.push_back(std::move(c));
  q->note_arrival(1 + n_votes);
  return COA_OK;
}

int coa_queue_submit_digest(coa_queue* q, const uint8_t* data, size_t len, coa_verdict_cb cb, void* user) {
  if (!q || (len && !data) || !cb) return COA_EINVAL;
  Dig d;
  d.data.assign(data, data + len);
  d.cb = cb;
  d.user = user;
  std::lock_guard<std::mutex> l(q->mu);
  if (q->stop) return COA_EINVAL;
  q->digs.push_back(std::move(d));
  q->note_arrival(1);
  return COA_OK;
}

int coa_queue_flush(coa_queue* q) {
  if (!q) return COA_EINVAL;
  std::unique_lock<std::mutex> l(q->mu);
  if (q->pending_sigs == 0 && !q->busy) return COA_OK;
  q->flush = true;
  q->cv.notify_one();
  q->idle_cv.wait(l, [&] { return q->pending_sigs == 0 && !q->busy; });
  return COA_OK;
}

int coa_queue_stats(coa_queue* q, uint64_t* launches, uint64_t* items, uint64_t* groups) {
  if (!q) return COA_EINVAL;
  std::lock_guard<std::mutex> l(q->mu);
  if (launches) *launches = q->launches;
  if (items) *items = q->items;
  if (groups) *groups = q->ngroups;
  return COA_OK;
}

int coa_queue_digest_count(coa_queue* q, uint64_t* digests) {
  if (!q || !digests) return COA_EINVAL;
  std::lock_guard<std::mutex> l(q->mu);
  *digests = q->ndigests;
  return COA_OK;
}

int coa_queue_destroy(coa_queue* q) {
  if (!q) return COA_EINVAL;
  coa_queue_flush(q);
  {
    std::lock_guard<std::mutex> l(q->mu);
    q->stop = true;
    q->cv.notify_one();
  }
  q->worker.join();
  delete q;
  return COA_OK;
}

}  // extern "C"
