// The engine's CPU path (csrc/coa_cpu.cpp, coa_cpu_*) under ASan + UBSan:
// every golden verify vector (any message length) one at a time and all at
// once on 4 threads, the golden batch groups with their weights, SHA-512 of
// the golden messages and a certificate round built from the vectors.  Input
// file (tests/test_sanitizers.py writes it): "CPUV" u32 n, then n records
// u32 msg_len | msg | pk | sig | u8 expect (1 = Ok); u32 groups, then per
// group msg(32) | u32 k | k x (pk | sig | z(16)) | u8 expect.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "coa_verify.h"

static bool rd(FILE* f, void* p, size_t n) { return fread(p, 1, n, f) == n; }

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  char magic[4];
  uint32_t n = 0;
  if (!rd(f, magic, 4) || memcmp(magic, "CPUV", 4) != 0 || !rd(f, &n, 4)) return 2;
  std::vector<std::vector<uint8_t>> msgs(n);
  std::vector<uint8_t> pks(32 * n), sigs(64 * n), expect(n);
  int bad = 0;
  for (uint32_t i = 0; i < n; i++) {
    uint32_t len = 0;
    if (!rd(f, &len, 4)) return 2;
    msgs[i].resize(len);
    if ((len && !rd(f, msgs[i].data(), len)) || !rd(f, &pks[32 * i], 32) || !rd(f, &sigs[64 * i], 64) ||
        !rd(f, &expect[i], 1))
      return 2;
    const int rc = coa_cpu_ed25519_verify_strict(msgs[i].data(), len, &pks[32 * i], &sigs[64 * i]);
    if ((rc == COA_OK) != (expect[i] == 1)) bad++;
  }
  // the 32-byte-message vectors in one many-call on 4 threads
  std::vector<uint8_t> m32, p32, s32, e32;
  for (uint32_t i = 0; i < n; i++)
    if (msgs[i].size() == 32) {
      m32.insert(m32.end(), msgs[i].begin(), msgs[i].end());
      p32.insert(p32.end(), &pks[32 * i], &pks[32 * i] + 32);
      s32.insert(s32.end(), &sigs[64 * i], &sigs[64 * i] + 64);
      e32.push_back(expect[i]);
    }
  std::vector<uint8_t> v(e32.size(), 9);
  if (coa_cpu_ed25519_verify_strict_many(m32.data(), 32, p32.data(), s32.data(), e32.size(), v.data(), 4) != COA_OK)
    bad++;
  for (size_t i = 0; i < e32.size(); i++)
    if ((v[i] == 0) != (e32[i] == 1)) bad++;
  // batch groups
  uint32_t groups = 0;
  if (!rd(f, &groups, 4)) return 2;
  for (uint32_t g = 0; g < groups; g++) {
    uint8_t msg[32], exp = 0;
    uint32_t k = 0;
    if (!rd(f, msg, 32) || !rd(f, &k, 4)) return 2;
    std::vector<uint8_t> gp(32 * k + 1), gs(64 * k + 1), gz(16 * k + 1);
    for (uint32_t j = 0; j < k; j++)
      if (!rd(f, &gp[32 * j], 32) || !rd(f, &gs[64 * j], 64) || !rd(f, &gz[16 * j], 16)) return 2;
    if (!rd(f, &exp, 1)) return 2;
    const uint64_t off[2] = {0, k};
    uint8_t gv = 9;
    if (coa_cpu_ed25519_verify_batch_groups_z(msg, gp.data(), gs.data(), off, 1, gz.data(), &gv, 1) != COA_OK ||
        (gv == 0) != (exp == 1))
      bad++;
  }
  fclose(f);
  // SHA-512 of every message, and certificates whose header input is the
  // message, id = its digest, header signature = the vector's signature,
  // no votes (each one's bits follow from the vector alone)
  std::vector<uint8_t> data;
  std::vector<uint64_t> offs{0};
  for (auto& m : msgs) {
    data.insert(data.end(), m.begin(), m.end());
    offs.push_back(data.size());
  }
  data.push_back(0);
  std::vector<uint8_t> d64(64 * (size_t)n);
  if (coa_cpu_sha512_many(data.data(), offs.data(), n, d64.data(), 3) != COA_OK) bad++;
  std::vector<uint8_t> ids(32 * (size_t)n), st(n, 9);
  for (uint32_t i = 0; i < n; i++) memcpy(&ids[32 * i], &d64[64 * i], 32);
  std::vector<uint64_t> rounds(n, 1), voff(n + 1, 0);
  if (coa_cpu_certificate_verify_many(data.data(), offs.data(), ids.data(), pks.data(), sigs.data(), rounds.data(),
                                      nullptr, nullptr, voff.data(), n, 5, st.data(), 4) != COA_OK)
    bad++;
  for (uint32_t i = 0; i < n; i++) {
    // bit 2 (header signature over the digest id) is the vector's own verdict
    // only when the vector signs that digest; just check the bit range
    if (st[i] & ~(uint8_t)(COA_CERT_BAD_HEADER_SIG)) bad++;
  }
  printf("cpu path ok: %u vectors, %u groups, %d bad\n", n, groups, bad);
  return bad != 0;
}
