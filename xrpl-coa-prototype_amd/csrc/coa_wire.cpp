// Wire decode of the primary's messages, host side.
//
// PrimaryReceiverHandler::dispatch (primary/src/primary.rs:223-244) runs
// `bincode::deserialize::<PrimaryMessage>` on every frame; Core then
// verifies one message at a time.  This decoder turns a window of frames into
// the struct-of-arrays the engine's batched entry points take (one
// coa_certificate_verify_many launch for all certificates of the window),
// without building per-message objects.
//
// Format: bincode 1.3 `deserialize` (legacy options: little-endian, fixed-
// width integers, u64 length prefixes, trailing bytes allowed) of
//   PrimaryMessage = u32 variant: 0 Header, 1 Vote, 2 Certificate,
//                    3 CertificatesRequest(Vec<Digest>, PublicKey)
//   Header      author PublicKey | round u64 | payload BTreeMap<Digest, u32>
//               | parents BTreeSet<Digest> | id Digest | signature
//   Vote        id | round u64 | origin PublicKey | author PublicKey | signature
//   Certificate header | votes Vec<(PublicKey, Signature)>
//   Digest      32 raw bytes;  Signature  part1 32 | part2 32
//   PublicKey   serde string (u64 length | UTF-8) holding base64 of the key
//               (crypto/src/lib.rs:94-112); decode_base64 keeps the first 32
//               decoded bytes (:72-78)
// (primary/src/messages.rs:13-21,105-112,168-172).  BTreeMap/BTreeSet
// deserialisation keeps the last value of a repeated key and iterates in key
// order, and Header::digest hashes that iteration (messages.rs:70-84), so the
// digest input emitted here is author | round LE | (digest | wid LE)* sorted |
// parents* sorted -- the bytes the reference hashes, not the wire bytes.
//
// Errors are per frame (the reference drops a frame whose decode fails).
// Where the reference would PANIC rather than error -- a base64 key that
// decodes to fewer than 32 bytes hits `bytes[..32]` at crypto/src/lib.rs:74
// -- this decoder reports COA_WIRE_EKEY instead.  base64 0.13 itself is not
// available here: canonical padded keys (what every node emits) are decoded
// exactly; for non-canonical forms this follows base64 0.13's documented
// STANDARD rules (padding optional, no bytes after padding, zero trailing
// bits) -- parity unpinned there.
#include <algorithm>
#include <array>
#include <cstring>
#include <map>
#include <set>
#include <vector>

#include "../../include/coa_verify.h"

namespace {

using D32 = std::array<uint8_t, 32>;

struct Rd {
  const uint8_t* p;
  size_t n, i = 0;
  bool ok = true;
  bool take(void* dst, size_t k) {
    if (!ok || n - i < k) return ok = false;
    if (dst) std::memcpy(dst, p + i, k);
    i += k;
    return true;
  }
  uint32_t u32() {
    uint32_t v = 0;
    take(&v, 4);
    return v;
  }
  uint64_t u64() {
    uint64_t v = 0;
    take(&v, 8);
    return v;
  }
};

int b64_val(uint8_t c) {
  if (c >= 'A' && c <= 'Z') return c - 'A';
  if (c >= 'a' && c <= 'z') return c - 'a' + 26;
  if (c >= '0' && c <= '9') return c - '0' + 52;
  if (c == '+') return 62;
  if (c == '/') return 63;
  return -1;
}

// base64 STANDARD decode; false on any malformed input.
bool b64_decode(const uint8_t* s, size_t len, std::vector<uint8_t>& out) {
  size_t body = len;
  while (body > 0 && s[body - 1] == '=') body--;
  const size_t pads = len - body;
  if (pads > 2) return false;
  if (body % 4 == 1) return false;
  if (pads && (body + pads) % 4 != 0) return false;
  out.clear();
  uint32_t acc = 0;
  int bits = 0;
  for (size_t i = 0; i < body; i++) {
    const int v = b64_val(s[i]);
    if (v < 0) return false;
    acc = (acc << 6) | (uint32_t)v;
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      out.push_back((uint8_t)(acc >> bits));
      acc &= (1u << bits) - 1;
    }
  }
  return acc == 0;  // trailing bits of the last symbol must be zero
}

// serde String: the bytes must be UTF-8 (structure check; a key is ASCII
// base64 anyway, so any non-ASCII byte fails one way or the other)
bool utf8_valid(const uint8_t* s, size_t n) {
  size_t i = 0;
  while (i < n) {
    const uint8_t c = s[i];
    size_t k;
    if (c < 0x80) k = 0;
    else if ((c >> 5) == 6) k = 1;
    else if ((c >> 4) == 14) k = 2;
    else if ((c >> 3) == 30) k = 3;
    else return false;
    if (n - i - 1 < k) return false;
    for (size_t j = 1; j <= k; j++)
      if ((s[i + j] & 0xC0) != 0x80) return false;
    i += k + 1;
  }
  return true;
}

int read_key(Rd& r, uint8_t out[32]) {
  const uint64_t len = r.u64();
  if (!r.ok || len > r.n - r.i) return COA_WIRE_ETRUNC;
  const uint8_t* s = r.p + r.i;
  r.i += len;
  if (!utf8_valid(s, len)) return COA_WIRE_EFORMAT;
  std::vector<uint8_t> bytes;
  if (!b64_decode(s, len, bytes)) return COA_WIRE_EKEY;
  if (bytes.size() < 32) return COA_WIRE_EKEY;  // the reference panics here
  std::memcpy(out, bytes.data(), 32);
  return COA_OK;
}

struct HeaderV {
  uint8_t author[32];
  uint64_t round;
  std::map<D32, uint32_t> payload;
  std::set<D32> parents;
  uint8_t id[32], sig[64];
};

int read_header(Rd& r, HeaderV& h) {
  int rc = read_key(r, h.author);
  if (rc != COA_OK) return rc;
  h.round = r.u64();
  const uint64_t np = r.u64();
  if (!r.ok || np > (r.n - r.i) / 36) return COA_WIRE_ETRUNC;
  for (uint64_t k = 0; k < np; k++) {
    D32 d;
    r.take(d.data(), 32);
    h.payload[d] = r.u32();  // BTreeMap: the last value of a repeated key wins
  }
  const uint64_t nq = r.u64();
  if (!r.ok || nq > (r.n - r.i) / 32) return COA_WIRE_ETRUNC;
  for (uint64_t k = 0; k < nq; k++) {
    D32 d;
    r.take(d.data(), 32);
    h.parents.insert(d);
  }
  r.take(h.id, 32);
  r.take(h.sig, 64);
  return r.ok ? COA_OK : COA_WIRE_ETRUNC;
}

size_t digest_input_len(const HeaderV& h) { return 40 + 36 * h.payload.size() + 32 * h.parents.size(); }

void digest_input(const HeaderV& h, uint8_t* out) {
  std::memcpy(out, h.author, 32);
  std::memcpy(out + 32, &h.round, 8);
  size_t o = 40;
  for (auto& kv : h.payload) {
    std::memcpy(out + o, kv.first.data(), 32);
    std::memcpy(out + o + 32, &kv.second, 4);
    o += 36;
  }
  for (auto& d : h.parents) {
    std::memcpy(out + o, d.data(), 32);
    o += 32;
  }
}

struct Frame {
  int kind = COA_WIRE_EFORMAT;
  HeaderV h;
  uint8_t vid[32], vorigin[32], vauthor[32], vsig[64];
  uint64_t vround = 0;
  std::vector<uint8_t> vote_pks, vote_sigs;
};

int parse(const uint8_t* p, size_t n, Frame& f) {
  Rd r{p, n};
  const uint32_t variant = r.u32();
  if (!r.ok) return f.kind = COA_WIRE_ETRUNC;
  int rc = COA_OK;
  switch (variant) {
    case 0:
      rc = read_header(r, f.h);
      break;
    case 1:
      r.take(f.vid, 32);
      f.vround = r.u64();
      if (!r.ok) return f.kind = COA_WIRE_ETRUNC;
      if ((rc = read_key(r, f.vorigin)) != COA_OK) break;
      if ((rc = read_key(r, f.vauthor)) != COA_OK) break;
      if (!r.take(f.vsig, 64)) rc = COA_WIRE_ETRUNC;
      break;
    case 2: {
      if ((rc = read_header(r, f.h)) != COA_OK) break;
      const uint64_t nv = r.u64();
      if (!r.ok || nv > (r.n - r.i) / (8 + 64)) {
        rc = COA_WIRE_ETRUNC;
        break;
      }
      f.vote_pks.resize(nv * 32);
      f.vote_sigs.resize(nv * 64);
      for (uint64_t k = 0; k < nv && rc == COA_OK; k++) {
        rc = read_key(r, &f.vote_pks[k * 32]);
        if (rc == COA_OK && !r.take(&f.vote_sigs[k * 64], 64)) rc = COA_WIRE_ETRUNC;
      }
      break;
    }
    case 3: {  // CertificatesRequest(Vec<Digest>, PublicKey): no crypto to do
      const uint64_t nd = r.u64();
      if (!r.ok || nd > (r.n - r.i) / 32) return f.kind = COA_WIRE_ETRUNC;
      r.take(nullptr, nd * 32);
      uint8_t k[32];
      rc = read_key(r, k);
      break;
    }
    default:
      return f.kind = COA_WIRE_EFORMAT;
  }
  return f.kind = (rc == COA_OK ? (int)variant : rc);
}

bool frames_ok(const uint8_t* frames, const uint64_t* offs, size_t n) {
  if (!offs) return false;
  for (size_t i = 0; i < n; i++)
    if (offs[i + 1] < offs[i]) return false;
  return !(offs[n] > offs[0] && !frames);
}

}  // namespace

extern "C" {

int coa_wire_scan(const uint8_t* frames, const uint64_t* frame_offsets, size_t n, int32_t* kind_out,
                  uint64_t* header_bytes_out, uint64_t* votes_out) {
  if (!kind_out || !frames_ok(frames, frame_offsets, n)) return COA_EINVAL;
  for (size_t i = 0; i < n; i++) {
    Frame f;
    kind_out[i] = parse(frames + frame_offsets[i], frame_offsets[i + 1] - frame_offsets[i], f);
    const bool hdr = kind_out[i] == COA_MSG_HEADER || kind_out[i] == COA_MSG_CERTIFICATE;
    if (header_bytes_out) header_bytes_out[i] = hdr ? digest_input_len(f.h) : 0;
    if (votes_out) votes_out[i] = kind_out[i] == COA_MSG_CERTIFICATE ? f.vote_pks.size() / 32 : 0;
  }
  return COA_OK;
}

int coa_wire_decode_certificates(const uint8_t* frames, const uint64_t* frame_offsets, size_t n, uint8_t* header_data,
                                 uint64_t* header_offsets, uint8_t* ids, uint8_t* origins, uint8_t* header_sigs,
                                 uint64_t* rounds, uint8_t* vote_pks, uint8_t* vote_sigs, uint64_t* vote_offsets,
                                 uint32_t* payload_counts) {
  if (!frames_ok(frames, frame_offsets, n) || !header_offsets || !ids || !origins || !header_sigs || !rounds ||
      !vote_offsets)
    return COA_EINVAL;
  header_offsets[0] = 0;
  vote_offsets[0] = 0;
  for (size_t i = 0; i < n; i++) {
    Frame f;
    if (parse(frames + frame_offsets[i], frame_offsets[i + 1] - frame_offsets[i], f) != COA_MSG_CERTIFICATE)
      return COA_EINVAL;  // coa_wire_scan first: only Certificate frames here
    const size_t hb = digest_input_len(f.h), nv = f.vote_pks.size() / 32;
    if (hb && !header_data) return COA_EINVAL;
    if (nv && (!vote_pks || !vote_sigs)) return COA_EINVAL;
    if (hb) digest_input(f.h, header_data + header_offsets[i]);
    header_offsets[i + 1] = header_offsets[i] + hb;
    std::memcpy(ids + i * 32, f.h.id, 32);
    std::memcpy(origins + i * 32, f.h.author, 32);
    std::memcpy(header_sigs + i * 64, f.h.sig, 64);
    rounds[i] = f.h.round;
    if (payload_counts) payload_counts[i] = (uint32_t)f.h.payload.size();
    if (nv) {
      std::memcpy(vote_pks + vote_offsets[i] * 32, f.vote_pks.data(), nv * 32);
      std::memcpy(vote_sigs + vote_offsets[i] * 64, f.vote_sigs.data(), nv * 64);
    }
    vote_offsets[i + 1] = vote_offsets[i] + nv;
  }
  return COA_OK;
}

int coa_wire_decode_votes(const uint8_t* frames, const uint64_t* frame_offsets, size_t n, uint8_t* ids,
                          uint64_t* rounds, uint8_t* origins, uint8_t* authors, uint8_t* sigs) {
  if (!frames_ok(frames, frame_offsets, n) || !ids || !rounds || !origins || !authors || !sigs) return COA_EINVAL;
  for (size_t i = 0; i < n; i++) {
    Frame f;
    if (parse(frames + frame_offsets[i], frame_offsets[i + 1] - frame_offsets[i], f) != COA_MSG_VOTE)
      return COA_EINVAL;
    std::memcpy(ids + i * 32, f.vid, 32);
    rounds[i] = f.vround;
    std::memcpy(origins + i * 32, f.vorigin, 32);
    std::memcpy(authors + i * 32, f.vauthor, 32);
    std::memcpy(sigs + i * 64, f.vsig, 64);
  }
  return COA_OK;
}

int coa_wire_decode_headers(const uint8_t* frames, const uint64_t* frame_offsets, size_t n, uint8_t* header_data,
                            uint64_t* header_offsets, uint8_t* ids, uint8_t* authors, uint8_t* sigs,
                            uint64_t* rounds, uint32_t* payload_counts) {
  if (!frames_ok(frames, frame_offsets, n) || !header_data || !header_offsets || !ids || !authors || !sigs ||
      !rounds)
    return COA_EINVAL;
  header_offsets[0] = 0;
  for (size_t i = 0; i < n; i++) {
    Frame f;
    if (parse(frames + frame_offsets[i], frame_offsets[i + 1] - frame_offsets[i], f) != COA_MSG_HEADER)
      return COA_EINVAL;
    const size_t hb = digest_input_len(f.h);
    digest_input(f.h, header_data + header_offsets[i]);
    header_offsets[i + 1] = header_offsets[i] + hb;
    std::memcpy(ids + i * 32, f.h.id, 32);
    std::memcpy(authors + i * 32, f.h.author, 32);
    std::memcpy(sigs + i * 64, f.h.sig, 64);
    rounds[i] = f.h.round;
    if (payload_counts) payload_counts[i] = (uint32_t)f.h.payload.size();
  }
  return COA_OK;
}

}  // extern "C"
