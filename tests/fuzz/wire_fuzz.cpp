// Mutation fuzzer of the native bincode decoder (xrpl-coa-prototype_amd/csrc/
// coa_wire.cpp), built with -fsanitize=address,undefined: the decoder parses
// untrusted network frames (the bytes PrimaryReceiverHandler::dispatch
// receives, primary/src/primary.rs:223-244), so every out-of-bounds read,
// overflow or UB on malformed input must be caught here.
//
// usage: wire_fuzz <corpus dir> <iterations> <seed>
// Each iteration mutates a batch of corpus frames -- truncation, byte flips,
// huge u64 length prefixes written at random offsets, bytes inserted or
// deleted, two frames spliced, base64 key characters replaced by invalid ones
// -- then runs coa_wire_scan on the batch and, for the frames it accepts,
// every decoder with output arrays sized exactly by the scan (so an overrun
// of the scan's own sizes is an ASan report).  Exit 0 when nothing fired.
#include <dirent.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <random>
#include <string>
#include <vector>

#include "coa_verify.h"

using Bytes = std::vector<uint8_t>;

static std::vector<Bytes> load(const std::string& dir) {
  std::vector<Bytes> out;
  DIR* d = opendir(dir.c_str());
  if (!d) return out;
  while (dirent* e = readdir(d)) {
    const std::string n = e->d_name;
    if (n.size() < 4 || n.substr(n.size() - 4) != ".bin") continue;
    std::ifstream f(dir + "/" + n, std::ios::binary);
    out.emplace_back(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
  }
  closedir(d);
  return out;
}

static Bytes mutate(const std::vector<Bytes>& corpus, std::mt19937_64& rng) {
  Bytes f = corpus[rng() % corpus.size()];
  const int rounds = 1 + (int)(rng() % 4);
  for (int r = 0; r < rounds; r++) {
    switch (rng() % 7) {
      case 0:  // truncate
        if (!f.empty()) f.resize(rng() % f.size());
        break;
      case 1:  // flip bytes
        for (int k = 0, m = 1 + (int)(rng() % 8); k < m && !f.empty(); k++) f[rng() % f.size()] ^= (uint8_t)(1 + rng() % 255);
        break;
      case 2: {  // a huge or off-by-a-little u64 length prefix at a random offset
        if (f.size() < 8) break;
        const size_t at = rng() % (f.size() - 7);
        static const uint64_t vals[] = {~0ull, 1ull << 62, 1ull << 32, 0xffffffffull, 1000000007ull, 33, 31, 0};
        const uint64_t v = vals[rng() % 8];
        std::memcpy(&f[at], &v, 8);
        break;
      }
      case 3: {  // insert random bytes
        const size_t at = f.empty() ? 0 : rng() % f.size();
        Bytes ins(1 + rng() % 40);
        for (auto& b : ins) b = (uint8_t)rng();
        f.insert(f.begin() + (long)at, ins.begin(), ins.end());
        break;
      }
      case 4:  // delete a range
        if (f.size() > 2) {
          const size_t a = rng() % f.size(), b = a + rng() % (f.size() - a);
          f.erase(f.begin() + (long)a, f.begin() + (long)b);
        }
        break;
      case 5: {  // splice with another frame
        const Bytes& g = corpus[rng() % corpus.size()];
        if (!f.empty() && !g.empty()) {
          f.resize(rng() % f.size());
          f.insert(f.end(), g.begin() + (long)(rng() % g.size()), g.end());
        }
        break;
      }
      default: {  // base64 alphabet violations where key strings usually sit
        static const char bad[] = {'=', '-', '_', '*', '\0', '\xff', ' ', '\n'};
        for (int k = 0, m = 1 + (int)(rng() % 3); k < m && !f.empty(); k++) f[rng() % f.size()] = (uint8_t)bad[rng() % 8];
        break;
      }
    }
  }
  return f;
}

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: wire_fuzz <corpus dir> <iterations> <seed>\n");
    return 2;
  }
  const std::vector<Bytes> corpus = load(argv[1]);
  if (corpus.empty()) {
    std::fprintf(stderr, "empty corpus\n");
    return 2;
  }
  const long iters = std::atol(argv[2]);
  std::mt19937_64 rng(std::strtoull(argv[3], nullptr, 10));
  long accepted[4] = {0, 0, 0, 0}, rejected = 0;
  for (long it = 0; it < iters; it++) {
    const size_t n = 1 + rng() % 8;
    std::vector<Bytes> fr(n);
    for (auto& f : fr) f = (it == 0) ? corpus[rng() % corpus.size()] : mutate(corpus, rng);
    // exact-size buffer per call (no slack, so ASan sees any overrun)
    Bytes buf;
    std::vector<uint64_t> off(n + 1, 0);
    for (size_t i = 0; i < n; i++) {
      buf.insert(buf.end(), fr[i].begin(), fr[i].end());
      off[i + 1] = buf.size();
    }
    uint8_t* data = (uint8_t*)std::malloc(buf.size() ? buf.size() : 1);
    if (!buf.empty()) std::memcpy(data, buf.data(), buf.size());
    std::vector<int32_t> kind(n);
    std::vector<uint64_t> hb(n), nv(n);
    if (coa_wire_scan(data, off.data(), n, kind.data(), hb.data(), nv.data()) != COA_OK) {
      std::fprintf(stderr, "scan refused a well-formed call\n");
      return 1;
    }
    for (size_t i = 0; i < n; i++) {
      if (kind[i] < 0) {
        rejected++;
        continue;
      }
      accepted[kind[i]]++;
      const uint64_t o[2] = {off[i], off[i + 1]};
      if (kind[i] == COA_MSG_CERTIFICATE) {
        std::vector<uint8_t> hd(hb[i] ? hb[i] : 1), ids(32), org(32), hs(64), vp(nv[i] * 32 + 1), vs(nv[i] * 64 + 1);
        uint64_t ho[2], rd[1], vo[2];
        uint32_t pc[1];
        const int rc = coa_wire_decode_certificates(data, o, 1, hd.data(), ho, ids.data(), org.data(), hs.data(), rd,
                                                    vp.data(), vs.data(), vo, pc);
        if (rc != COA_OK || ho[1] != hb[i] || vo[1] != nv[i]) {
          std::fprintf(stderr, "certificate decode disagrees with its scan (rc %d)\n", rc);
          return 1;
        }
      } else if (kind[i] == COA_MSG_HEADER) {
        std::vector<uint8_t> hd(hb[i] ? hb[i] : 1), ids(32), au(32), sg(64);
        uint64_t ho[2], rd[1];
        uint32_t pc[1];
        const int rc = coa_wire_decode_headers(data, o, 1, hd.data(), ho, ids.data(), au.data(), sg.data(), rd, pc);
        if (rc != COA_OK || ho[1] != hb[i]) {
          std::fprintf(stderr, "header decode disagrees with its scan (rc %d)\n", rc);
          return 1;
        }
      } else if (kind[i] == COA_MSG_VOTE) {
        std::vector<uint8_t> ids(32), org(32), au(32), sg(64);
        uint64_t rd[1];
        const int rc = coa_wire_decode_votes(data, o, 1, ids.data(), rd, org.data(), au.data(), sg.data());
        if (rc != COA_OK) {
          std::fprintf(stderr, "vote decode failed after a good scan (rc %d)\n", rc);
          return 1;
        }
      }
    }
    std::free(data);
  }
  std::printf("wire fuzz ok: %ld iterations, accepted header %ld vote %ld certificate %ld request %ld, rejected %ld\n",
              iters, accepted[0], accepted[1], accepted[2], accepted[3], rejected);
  return 0;
}
