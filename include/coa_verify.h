/*
 * coa_verify.h -- C ABI of the MI355X (gfx950) ed25519 / SHA-512 verification
 * engine for the Narwhal/Tusk fork pwang200/xrpl-coa-prototype.
 *
 * This is the drop-in boundary for the reference's `crypto` crate hot path.
 * Every entry point names the reference interface it replaces.  Plain
 * pointers and sizes only: no HIP or torch types in the signatures (device
 * streams are passed as `void*` = hipStream_t).
 *
 * Conventions
 *   - Verdict bytes: 0 = Ok, 1 = Err (the reference's Result<(), CryptoError>;
 *     CryptoError = ed25519::Error is opaque, crypto/src/lib.rs:18, so callers
 *     only branch Ok/Err -- primary/src/error.rs:28 maps it to
 *     DagError::InvalidSignature).
 *   - Return codes: COA_OK (0) / COA_REJECT (1) for single verdicts; COA_OK for
 *     a completed many-call; a negative COA_E* on internal failure.  There is
 *     NO implicit CPU fallback: with no usable GPU every GPU call returns
 *     COA_ENODEVICE.  The engine's own CPU path (coa_cpu_*, below) answers
 *     only when a caller calls it explicitly.
 *   - Host-pointer calls: inputs are caller-owned and only read during the
 *     call; outputs are caller-allocated.  Nothing is retained after return.
 *   - Thread safety: every call takes the engine lock of the devices it uses;
 *     calls from several threads are serialised per device.
 *   - Multi-GPU: host-pointer "many" calls shard items by contiguous index
 *     range over the devices opened by coa_init (no cross-GPU exchange).
 */
#ifndef COA_VERIFY_H
#define COA_VERIFY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define COA_OK 0
#define COA_REJECT 1
#define COA_EINVAL (-1)
#define COA_ENODEVICE (-2)
#define COA_EHIP (-3)
#define COA_ENOMEM (-4)

/* ---------------------------------------------------------------- lifecycle
 * No reference counterpart (dalek is stateless).  Opens `n_gpus` devices
 * (0 = all visible), builds the fixed-base tables on each.  Idempotent; the
 * other calls initialise lazily with n_gpus = 0 when it was not called. */
int coa_init(int n_gpus);
/* Opens exactly the listed HIP devices (one process per GPU: each rank opens
 * its own).  Idempotent like coa_init; host-pointer calls shard over the
 * opened devices in list order. */
int coa_init_devices(const int* device_ids, int n);
int coa_shutdown(void);
int coa_device_count(void);
/* HIP device id of each opened context, in the order host-pointer calls
 * shard over them (a device opened k times appears k times).  Returns the
 * number of contexts; copies min(count, cap) ids. */
int coa_device_ids(int* ids_out, int cap);
/* Self-test of device `device`'s fixed-base tables (no reference
 * counterpart): checks every entry of the wide HBM comb of B against its
 * neighbours (m*2^(Wj)*B = (m-1)*2^(Wj)*B + 2^(Wj)*B, 2^(W(j+1))*B =
 * [2^W] 2^(Wj)*B, entry (0,1) = B, canonical encodings).  *bad_entries gets
 * the number of failing entries (0 when the table is absent: COA_WCOMB=0). */
int coa_self_test(int device, uint64_t* bad_entries);
/* Self-test of the row-parallel field arithmetic (no reference counterpart):
 * for each of the n 32-byte values d_in[i] (device memory, any value below
 * 2^256) compares, on the device, the 16-lane-row versions of z^((p-5)/8),
 * z^(p-2), z * d_in[i+1], z + d_in[i+1], z - d_in[i+1] and decompression (of
 * d_in[i] as an encoding) with
 * the one-lane versions.  d_out[i] (uint32) gets a bit per mismatch: 0 = agree.
 * stream NULL = the engine's stream (the call then waits). */
int coa_fe_rows_check_device(int device, const uint8_t* d_in, size_t n, uint32_t* d_out, void* stream);
/* Human-readable description of the last error on this thread. */
const char* coa_last_error(void);
/* Engine-failure recovery of the host-pointer calls since the library
 * loaded (no reference counterpart: dalek cannot fail for a reason other
 * than the input).  A shard whose device work fails (a HIP error or an
 * allocation failure) has its context rebuilt -- a new stream, per-call
 * buffers released, in the same process -- and is re-run on the next
 * contexts in turn; the call returns an error only when every context
 * failed it.  *contexts_rebuilt / *shards_rerun (either may be NULL) get the
 * counts.  The aggregation queue counts its own in coa_queue_metrics. */
int coa_engine_recoveries(uint64_t* contexts_rebuilt, uint64_t* shards_rerun);
/* Library / ABI version string. */
const char* coa_version(void);

/* ------------------------------------------------------- Signature::verify
 * Replaces crypto::Signature::verify (crypto/src/lib.rs:200-204):
 *   ed25519::Signature::from_bytes(sig)            (:201)
 *   ed25519_dalek::PublicKey::from_bytes(pk)       (:202)
 *   PublicKey::verify_strict(msg, sig)             (:203)
 * called by Header::verify (primary/src/messages.rs:64-66) and Vote::verify
 * (primary/src/messages.rs:139-141).  msg is the 32-byte Digest.
 * Returns COA_OK, COA_REJECT or a negative error (latency path). */
int coa_ed25519_verify_strict(const uint8_t msg[32], const uint8_t pk[32], const uint8_t sig[64]);

/* n independent (msg, pk, sig) triples; msgs are n * msg_len bytes (msg_len
 * 32 for the crypto API, any length supported), pks n * 32, sigs n * 64
 * (R || s).  verdicts_out[i] = 0 Ok / 1 Err.  Sharded over all devices. */
int coa_ed25519_verify_strict_many(const uint8_t* msgs, size_t msg_len, const uint8_t* pks, const uint8_t* sigs,
                                   size_t n, uint8_t* verdicts_out);

/* Same, with every buffer already resident in the HBM of `device` and the
 * work enqueued on `stream` (hipStream_t; NULL = the engine's stream for that
 * device).  Asynchronous: returns after enqueue.  `workspace` may be NULL
 * (engine-owned) -- otherwise at least coa_verify_workspace_bytes(n) bytes of
 * device memory on `device`. */
size_t coa_verify_workspace_bytes(size_t n);
int coa_ed25519_verify_strict_many_device(int device, const uint8_t* d_msgs, size_t msg_len, const uint8_t* d_pks,
                                          const uint8_t* d_sigs, size_t n, uint8_t* d_verdicts, void* workspace,
                                          void* stream);

/* The two device stages of the call above, for callers that already hold k
 * (e.g. a digest stage fused upstream) and for per-kernel timing:
 *   challenge:  d_k_out[i] = SHA-512(R_i || A_i || M_i) mod l, 32 bytes LE
 *               (Scalar::from_hash inside dalek verify_strict)
 *   prehashed:  verdicts from (k, A, R || s); workspace as above (may be NULL). */
int coa_ed25519_challenge_many_device(int device, const uint8_t* d_msgs, size_t msg_len, const uint8_t* d_pks,
                                      const uint8_t* d_sigs, size_t n, uint8_t* d_k_out, void* stream);
int coa_ed25519_verify_prehashed_many_device(int device, const uint8_t* d_k, const uint8_t* d_pks,
                                             const uint8_t* d_sigs, size_t n, uint8_t* d_verdicts, void* workspace,
                                             void* stream);

/* ------------------------------------------------- Signature::verify_batch
 * Replaces crypto::Signature::verify_batch (crypto/src/lib.rs:206-219) ->
 * ed25519_dalek::verify_batch (:218), called by Certificate::verify
 * (primary/src/messages.rs:214).  One group = one certificate: all its votes
 * sign the same 32-byte digest.
 *   msgs           n_groups * 32 bytes
 *   pks, sigs      concatenated votes, group g = [group_offsets[g], group_offsets[g+1])
 *   group_offsets  n_groups + 1 entries, group_offsets[0] = 0
 *   group_verdicts_out[g] = 0 Ok / 1 Err
 * The 128-bit random weights z_i are derived from rng_seed (0 = fresh OS
 * entropy per call, the dalek behaviour; any other value is reproducible).
 * Ok iff every s_i < l, every A_i and R_i decompresses and the random linear
 * combination is the identity -- no small-order rejection, no cofactor,
 * exactly dalek 1.0.1. */
int coa_ed25519_verify_batch(const uint8_t msg[32], const uint8_t* pks, const uint8_t* sigs, size_t n,
                             uint64_t rng_seed);
int coa_ed25519_verify_batch_groups(const uint8_t* msgs, const uint8_t* pks, const uint8_t* sigs,
                                    const uint64_t* group_offsets, size_t n_groups, uint8_t* group_verdicts_out,
                                    uint64_t rng_seed);
/* Parity-test form: the z_i are given explicitly (16 little-endian bytes per
 * signature, in the order of pks/sigs). */
int coa_ed25519_verify_batch_groups_z(const uint8_t* msgs, const uint8_t* pks, const uint8_t* sigs,
                                      const uint64_t* group_offsets, size_t n_groups, const uint8_t* zs,
                                      uint8_t* group_verdicts_out);

/* Pippenger form of the call above for ONE group whose buffers are resident
 * in the HBM of `device` (dalek's verify_batch switches to Pippenger above
 * 190 points; the host-pointer entries above route here the groups of a
 * call with one or two groups, and groups of at least COA_MSM_MIN
 * signatures, default 16384).
 *   d_msg        32 bytes, the digest every signature signs
 *   d_pks        n * 32, d_sigs n * 64
 *   d_zs         n * 16 explicit weights (parity tests) or NULL = derived
 *                from rng_seed (0 = fresh OS entropy)
 *   *d_verdict   0 Ok / 1 Err, same rules as coa_ed25519_verify_batch
 * `workspace` NULL = engine-owned (the call then waits for the stream), else
 * `workspace_bytes` bytes on `device`, at least
 * coa_verify_batch_workspace_bytes(n) evaluated under the same environment
 * (COA_MSM_RUN changes the layout); a smaller buffer is refused with
 * COA_EINVAL.  With a workspace the call only enqueues. */
size_t coa_verify_batch_workspace_bytes(size_t n);
int coa_ed25519_verify_batch_device(int device, const uint8_t* d_msg, const uint8_t* d_pks, const uint8_t* d_sigs,
                                    size_t n, const uint8_t* d_zs, uint64_t rng_seed, uint8_t* d_verdict,
                                    void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------ Digest
 * Replaces Sha512::digest at worker/src/processor.rs:38 (500 KB batch
 * digests) and the Header/Vote/Certificate digests
 * (primary/src/messages.rs:70-84,145-153,226-234).  Message i is
 * data[offsets[i] .. offsets[i+1]); offsets has n + 1 entries.
 * coa_sha512_many writes 64 bytes per message, coa_sha512_trunc32_many the
 * 32-byte crypto::Digest prefix. */
int coa_sha512_many(const uint8_t* data, const uint64_t* offsets, size_t n, uint8_t* out64);
int coa_sha512_trunc32_many(const uint8_t* data, const uint64_t* offsets, size_t n, uint8_t* out32);
int coa_sha512_many_device(int device, const uint8_t* d_data, const uint64_t* d_offsets, size_t n, uint8_t* d_out64,
                           void* stream);

/* ------------------------------------------------ committee key cache (f2)
 * No reference counterpart: the reference decompresses every voter key on
 * every call (crypto/src/lib.rs:202,216) although the keys are fixed per
 * config::Committee (config/src/lib.rs:140-143, loaded once in
 * node/src/main.rs).  Registers the committee's n public keys (32 B each;
 * duplicates collapse) on every device: decompression verdict, small-order
 * and torsion flags and a 384 KiB comb of -A per key, so certificate checks
 * need no doubling.  Replaces any previous committee; n = 0 clears it.
 * Verdict-neutral: keys outside the committee still verify, through the
 * uncached kernels.  Returns the number of distinct keys registered or a
 * negative error. */
int coa_committee_register(const uint8_t* pks, size_t n);
/* Key flags of the registered committee in its internal (sorted) order:
 * bit0 decompresses, bit1 small order, bit2 torsion free.  Returns the
 * committee size; copies min(size, cap) words.  Diagnostics / tests. */
int coa_committee_key_flags(uint32_t* flags_out, size_t cap);

/* --------------------------------------- Certificate::verify crypto (f3)
 * The crypto of Certificate::verify (primary/src/messages.rs:189-215) in one
 * fused launch for registered committees:
 *   COA_CERT_BAD_HEADER_ID   SHA-512(header digest bytes)[..32] != header.id
 *                            (Header::verify, messages.rs:49-51; the bytes are
 *                            Header::digest's input, messages.rs:70-84)
 *   COA_CERT_BAD_HEADER_SIG  Signature::verify(header.id, author) fails
 *                            (messages.rs:64-66, dalek verify_strict)
 *   COA_CERT_BAD_VOTES       Signature::verify_batch(Certificate::digest,
 *                            votes) fails (messages.rs:214; the digest is
 *                            SHA-512(id || round u64 LE || origin)[..32],
 *                            messages.rs:226-234, computed on the device)
 * The non-crypto checks (genesis, stake, worker ids, quorum) stay with the
 * caller, which applies them in the reference's order with these bits
 * (INTEGRATION.md).  Votes are checked per signature with the committee
 * combs; when every vote holds its own cofactorless equation and every key is
 * torsion free, dalek's batch verdict is Ok for any weights.  Any other
 * well-formed outcome is re-decided by the exact random-linear-combination
 * kernels (weights from rng_seed, 0 = OS entropy, as verify_batch), and
 * certificates with keys outside the committee take the uncached kernels:
 * the verdict is always dalek's.
 *   header_data/header_offsets  n + 1 offsets into the concatenated headers
 *   ids, origins                n * 32 (header.id, header.author)
 *   header_sigs                 n * 64;  rounds: n
 *   vote_pks, vote_sigs         concatenated votes; certificate c owns
 *                               [vote_offsets[c], vote_offsets[c+1])
 *   status_out[c]               0 = all crypto Ok, else COA_CERT_* bits */
#define COA_CERT_BAD_HEADER_ID 1
#define COA_CERT_BAD_HEADER_SIG 2
#define COA_CERT_BAD_VOTES 4
int coa_certificate_verify_many(const uint8_t* header_data, const uint64_t* header_offsets, const uint8_t* ids,
                                const uint8_t* origins, const uint8_t* header_sigs, const uint64_t* rounds,
                                const uint8_t* vote_pks, const uint8_t* vote_sigs, const uint64_t* vote_offsets,
                                size_t n, uint64_t rng_seed, uint8_t* status_out);
/* One certificate (the latency path: one H2D, one launch with one wavefront
 * per signature, one D2H).  Returns the COA_CERT_* bits (>= 0) or a negative
 * error. */
int coa_certificate_verify(const uint8_t* header_data, size_t header_len, const uint8_t id[32],
                           const uint8_t origin[32], const uint8_t header_sig[64], uint64_t round,
                           const uint8_t* vote_pks, const uint8_t* vote_sigs, size_t n_votes, uint64_t rng_seed);
/* Device-resident form (asynchronous on `stream`): d_status[c] receives the
 * raw status word -- COA_CERT_* bits plus 8 = votes need the exact RLC check
 * (coa_ed25519_verify_batch_groups) and 16 = a key is not registered (use the
 * uncached entry points).  The host-pointer calls above resolve both.
 * `workspace`: NULL (engine-owned; the call then waits for its stream) or
 * coa_certificate_workspace_bytes(n, n_votes) bytes of device memory.  A
 * call of >= 16,384 jobs (certificates + votes) takes its jobs in committee-key
 * order, and the size then includes the sort's area (~4.2 MB + 8 B per job). */
size_t coa_certificate_workspace_bytes(size_t n, size_t n_votes);
int coa_certificate_verify_many_device(int device, const uint8_t* d_header_data, const uint64_t* d_header_offsets,
                                       const uint8_t* d_ids, const uint8_t* d_origins, const uint8_t* d_header_sigs,
                                       const uint64_t* d_rounds, const uint8_t* d_vote_pks,
                                       const uint8_t* d_vote_sigs, const uint64_t* d_vote_offsets, size_t n,
                                       size_t n_votes, uint32_t* d_status, void* workspace, void* stream);

/* ------------------------------------------------------- wire decode (f4)
 * bincode 1.3 decode of PrimaryMessage frames, as
 * PrimaryReceiverHandler::dispatch does (primary/src/primary.rs:223-244),
 * straight into the arrays of the batched entry points above.  Host-only
 * parsing (no device work).  frames[frame_offsets[i] .. frame_offsets[i+1])
 * is frame i.
 *   coa_wire_scan: kind_out[i] = COA_MSG_* or a negative COA_WIRE_E* (the
 *     reference drops such frames); header_bytes_out[i] = length of the
 *     Header::digest input (Header and Certificate frames), votes_out[i] =
 *     number of votes (Certificate frames); both optional.
 *   coa_wire_decode_certificates: every frame must be a Certificate; fills
 *     the coa_certificate_verify_many arguments (header_data sized by the
 *     scan's header bytes, vote arrays by its vote counts); payload_counts
 *     (optional) = entries of header.payload, whose worker ids sit at
 *     header_data + 40 + 36 k + 32 (the MalformedHeader check).
 *   coa_wire_decode_votes / _headers: Vote / Header frames (Vote::digest
 *     input = id || round LE || origin; Header::digest input as above).
 * Header::digest input = author | round LE | (digest | worker id LE)* in key
 * order | parents* in order (primary/src/messages.rs:70-84). */
#define COA_MSG_HEADER 0
#define COA_MSG_VOTE 1
#define COA_MSG_CERTIFICATE 2
#define COA_MSG_CERT_REQUEST 3
#define COA_WIRE_ETRUNC (-10)  /* frame ends inside a field / length prefix too large */
#define COA_WIRE_EFORMAT (-11) /* unknown variant or non-UTF-8 string */
#define COA_WIRE_EKEY (-12)    /* PublicKey string is not base64 of >= 32 bytes */
int coa_wire_scan(const uint8_t* frames, const uint64_t* frame_offsets, size_t n, int32_t* kind_out,
                  uint64_t* header_bytes_out, uint64_t* votes_out);
int coa_wire_decode_certificates(const uint8_t* frames, const uint64_t* frame_offsets, size_t n, uint8_t* header_data,
                                 uint64_t* header_offsets, uint8_t* ids, uint8_t* origins, uint8_t* header_sigs,
                                 uint64_t* rounds, uint8_t* vote_pks, uint8_t* vote_sigs, uint64_t* vote_offsets,
                                 uint32_t* payload_counts);
int coa_wire_decode_votes(const uint8_t* frames, const uint64_t* frame_offsets, size_t n, uint8_t* ids,
                          uint64_t* rounds, uint8_t* origins, uint8_t* authors, uint8_t* sigs);
int coa_wire_decode_headers(const uint8_t* frames, const uint64_t* frame_offsets, size_t n, uint8_t* header_data,
                            uint64_t* header_offsets, uint8_t* ids, uint8_t* authors, uint8_t* sigs,
                            uint64_t* rounds, uint32_t* payload_counts);

/* --------------------------------------------------------------- signing
 * RFC 8032 signing == crypto::Signature::new (crypto/src/lib.rs:185-191) /
 * generate_keypair (:167-175) from 32-byte seeds.  Not on the verification
 * hot path; used to synthesise benchmark and test inputs on the device. */
int coa_ed25519_public_keys(const uint8_t* seeds, size_t n, uint8_t* pks_out);
int coa_ed25519_sign_many(const uint8_t* seeds, const uint8_t* msgs, size_t msg_len, size_t n, uint8_t* pks_out,
                          uint8_t* sigs_out);
int coa_ed25519_sign_many_device(int device, const uint8_t* d_seeds, const uint8_t* d_msgs, size_t msg_len, size_t n,
                                 uint8_t* d_pks_out, uint8_t* d_sigs_out, void* stream);

/* ------------------------------------------ the engine's own CPU path
 * The same checks as the GPU entry points above, on the host's cores
 * (csrc/coa_cpu.cpp; dalek 1.0.1 acceptance rules, verdict for verdict).
 * NEVER called implicitly: a GPU entry point that cannot answer returns a
 * negative COA_E*.  A caller that must keep answering calls these explicitly
 * -- the Rust binding does under COA_ON_ENGINE_FAILURE=cpu
 * (rust/crypto/src/degrade.rs), so verdicts do not depend on device health
 * (SURVEY.md §5).  nthreads <= 0: min(16, hardware threads).  Same return
 * conventions as the GPU forms; no coa_init needed.
 *   coa_cpu_ed25519_verify_strict      crypto/src/lib.rs:200-204
 *   coa_cpu_ed25519_verify_batch[_groups_z]  crypto/src/lib.rs:206-219
 *                                      (rng_seed as coa_ed25519_verify_batch)
 *   coa_cpu_sha512_many                worker/src/processor.rs:38,
 *                                      primary/src/messages.rs:70-84,226-234
 *   coa_cpu_certificate_verify_many[_z]  primary/src/messages.rs:189-215
 *                                      (status_out: COA_CERT_* bits; _z takes
 *                                      the votes' 16-byte weights) */
int coa_cpu_ed25519_verify_strict(const uint8_t* msg, size_t msg_len, const uint8_t pk[32], const uint8_t sig[64]);
int coa_cpu_ed25519_verify_strict_many(const uint8_t* msgs, size_t msg_len, const uint8_t* pks, const uint8_t* sigs,
                                       size_t n, uint8_t* verdicts_out, int nthreads);
int coa_cpu_ed25519_verify_batch(const uint8_t msg[32], const uint8_t* pks, const uint8_t* sigs, size_t n,
                                 uint64_t rng_seed);
int coa_cpu_ed25519_verify_batch_groups_z(const uint8_t* msgs, const uint8_t* pks, const uint8_t* sigs,
                                          const uint64_t* group_offsets, size_t n_groups, const uint8_t* zs,
                                          uint8_t* group_verdicts_out, int nthreads);
int coa_cpu_sha512_many(const uint8_t* data, const uint64_t* offsets, size_t n, uint8_t* out64, int nthreads);
int coa_cpu_certificate_verify_many(const uint8_t* header_data, const uint64_t* header_offsets, const uint8_t* ids,
                                    const uint8_t* origins, const uint8_t* header_sigs, const uint64_t* rounds,
                                    const uint8_t* vote_pks, const uint8_t* vote_sigs, const uint64_t* vote_offsets,
                                    size_t n, uint64_t rng_seed, uint8_t* status_out, int nthreads);
int coa_cpu_certificate_verify_many_z(const uint8_t* header_data, const uint64_t* header_offsets, const uint8_t* ids,
                                      const uint8_t* origins, const uint8_t* header_sigs, const uint64_t* rounds,
                                      const uint8_t* vote_pks, const uint8_t* vote_sigs, const uint64_t* vote_offsets,
                                      size_t n, const uint8_t* zs, uint8_t* status_out, int nthreads);

/* ------------------------------------------------ aggregation queue (f1)
 * Pre-verification stage for Core::run (primary/src/core.rs:349-389), which
 * verifies one message at a time: producers submit header/vote signatures,
 * vote batches, certificates and worker batch digests; the queue coalesces
 * them into launches (when max_batch items are pending, when the oldest
 * request is max_delay_us old, or on flush) and replies per request through
 * the callback -- the SignatureService request/oneshot idiom of
 * crypto/src/lib.rs:222-250.  Inputs are copied at submission (into one of
 * a fixed pool of intake shards, chosen by the calling thread).  Two lanes,
 * each with its own collector, device slots and completion thread: one for
 * signatures, vote batches and certificates, one for digests (a digest
 * window is a 14 ms serial chain; it never delays a verdict).  A lane's
 * collector launches each window on a free slot (four per GPU for verdicts,
 * eight for digests, COA_QUEUE_SLOTS / COA_QUEUE_DIGEST_SLOTS; pinned staging, its own stream
 * on its own hardware queue, COA_QUEUE_STREAMS) without waiting for the
 * previous window, and its completion thread answers windows in order: the
 * callback runs there with status (COA_OK or a negative engine error) and
 * the request's verdict byte(s).  The requests a window's kernels cannot
 * decide alone -- certificates with a key outside the registered committee
 * or with votes that failed their own equation, and bare vote batches -- are
 * answered later, by the lane's resolver thread (the exact path), so they
 * never hold back the rest of their window; answers are therefore not in
 * submission order across requests.  Windows that read the committee key cache
 * pin the generation they launched with; coa_committee_register builds the
 * next generation beside it, so registration neither waits for nor holds
 * back a window and stays verdict-neutral under load. */
typedef struct coa_queue coa_queue;
typedef void (*coa_verdict_cb)(void* user, int status, const uint8_t* verdicts, size_t n);
coa_queue* coa_queue_create(size_t max_batch, uint32_t max_delay_us);
int coa_queue_submit_verify(coa_queue* q, const uint8_t msg[32], const uint8_t pk[32], const uint8_t sig[64],
                            coa_verdict_cb cb, void* user);
/* n independent triples in one request (one copy, one lock, one callback
 * with the n verdict bytes in order): for producers that already hold a
 * group of messages, e.g. a window of received votes. */
int coa_queue_submit_verify_many(coa_queue* q, const uint8_t* msgs, const uint8_t* pks, const uint8_t* sigs, size_t n,
                                 coa_verdict_cb cb, void* user);
int coa_queue_submit_batch(coa_queue* q, const uint8_t msg[32], const uint8_t* pks, const uint8_t* sigs, size_t n,
                           coa_verdict_cb cb, void* user);
/* Whole certificates (the fused Certificate::verify crypto, f3): the
 * callback receives one status byte of COA_CERT_* bits (0 = all Ok). */
int coa_queue_submit_certificate(coa_queue* q, const uint8_t* header_data, size_t header_len, const uint8_t id[32],
                                 const uint8_t origin[32], const uint8_t header_sig[64], uint64_t round,
                                 const uint8_t* vote_pks, const uint8_t* vote_sigs, size_t n_votes, coa_verdict_cb cb,
                                 void* user);
/* The same without the copy: the arrays are read in place -- packed by the
 * launch that takes the request straight into the device staging, and read
 * again by the resolver if the certificate needs the exact re-decision -- so
 * they must stay valid and unchanged until the callback has run.  For callers
 * that hold each request's bytes until its answer anyway
 * (rust/crypto/src/service.rs boxes them with the reply sender): the
 * producer's copy, one of the streamed path's two host copies, is gone. */
int coa_queue_submit_certificate_borrowed(coa_queue* q, const uint8_t* header_data, size_t header_len,
                                          const uint8_t id[32], const uint8_t origin[32], const uint8_t header_sig[64],
                                          uint64_t round, const uint8_t* vote_pks, const uint8_t* vote_sigs,
                                          size_t n_votes, coa_verdict_cb cb, void* user);
/* Worker batch digests (worker/src/processor.rs:38, Processor::spawn): the
 * callback receives the 32-byte Digest (n = 32). */
int coa_queue_submit_digest(coa_queue* q, const uint8_t* data, size_t len, coa_verdict_cb cb, void* user);
int coa_queue_flush(coa_queue* q);
/* Window policy (no reference counterpart): with windows_in_flight = k > 0 a
 * window also closes at once while fewer than k windows are in flight, so a
 * request reaching an idle queue launches without waiting out max_delay_us;
 * under load requests still coalesce behind the windows in flight.  0 (the
 * default; COA_QUEUE_IDLE_LAUNCH=k at creation sets k) keeps the deadline
 * policy alone.  For latency-bound stages (the primary's pre-verification:
 * committee-100 round mix p50 0.31-0.39 -> 0.07-0.26 ms) rather than
 * throughput streams (worker batch digests). */
int coa_queue_set_idle_launch(coa_queue* q, uint32_t windows_in_flight);
/* items = signatures answered (a coa_queue_submit_verify_many request of n
 * counts n); groups = vote batches + certificates. */
int coa_queue_stats(coa_queue* q, uint64_t* launches, uint64_t* items, uint64_t* groups);
int coa_queue_digest_count(coa_queue* q, uint64_t* digests);
/* Queue metrics since creation.  A window is the set of requests one launch
 * takes; windows are pipelined (the next window is packed and its copies and
 * kernels enqueued while the previous one runs).  wait_us_* is the time from
 * a request's submission to the start of its callback (percentiles from a
 * log-spaced histogram, +-6 %).
 * Engine-failure recovery: a window whose launch fails (a HIP error) is
 * re-run on the recovery context of each device in turn (the failed slot's
 * stream, event and buffers rebuilt meanwhile, in the same process); its
 * callbacks get a negative status only when every attempt failed. */
typedef struct {
  uint64_t requests;      /* requests answered */
  uint64_t windows;       /* launch windows */
  uint64_t signatures;    /* signatures answered (verify requests x their n) */
  uint64_t batches;       /* vote-batch requests */
  uint64_t certificates;  /* certificate requests */
  uint64_t digests;       /* digest requests */
  uint64_t max_window;    /* most items (signatures + votes + digests) in one window */
  uint64_t max_in_flight; /* most windows launched and not yet answered at once */
  uint64_t max_pending;   /* most items waiting for a window at once */
  double wait_us_mean, wait_us_p50, wait_us_p99, wait_us_max;
  uint64_t retried_windows;   /* windows whose launch failed and were re-run */
  uint64_t recovered_windows; /* ... of which a re-run succeeded */
  uint64_t failed_windows;    /* windows answered with an engine error */
  /* where a tail comes from: the slowest window from its launch call (the
   * collector hands it to a slot) to its outputs in host memory, with its
   * size and kinds; the longest a launch waited for a free slot; staging
   * reallocations (page-locked or device allocations on the launch path) */
  double window_us_max;
  uint64_t window_max_items;
  uint32_t window_max_kinds;  /* COA_QUEUE_KIND_* bits */
  int32_t stream_kind;        /* COA_QUEUE_STREAM_*: how the slots' streams were made */
  double slot_wait_us_max;
  uint64_t staging_grows;     /* windows that had to enlarge a slot's staging or workspace (warm-up not counted) */
  uint32_t slots_verify, slots_digest; /* device slots of each lane, over all devices */
  /* Two-step answers: certificates the fused kernel could not decide alone
   * (a key outside the registered committee, an inconclusive vote) and bare
   * vote batches go to the lane's resolver thread, which decides them exactly
   * (coa_certificate_verify_many's semantics); the rest of their window is
   * answered at once.  So one open certificate never holds back the requests
   * it shares a window with, nor the windows behind it. */
  uint64_t deferred_requests; /* requests answered by the resolver */
  uint64_t resolver_passes;   /* resolver passes (each decides every open request queued by then) */
  double resolve_us_max;      /* the longest resolver pass */
  /* Where the time goes, summed over every window (microseconds, COA_QSTAGE_*
   * indices; divide by `windows` for a mean per window). */
  double stage_us[12];
  /* When the slowest window (window_us_max) was launched, in milliseconds
   * since the queue's creation or its last coa_queue_metrics_reset, and how
   * much of it was spent waiting for its device work (COA_QSTAGE_DEVICE_WAIT):
   * a one-off tail at a run's start points at set-up costs, one in the
   * device wait at the device. */
  double window_max_at_ms;
  double window_max_device_us;
} coa_queue_metrics_t;
#define COA_QSTAGE_INTAKE 0      /* producers: shard lock + copy of the request into the shard */
#define COA_QSTAGE_GATHER 1      /* collector: taking the shards' windows */
#define COA_QSTAGE_SLOT_WAIT 2   /* launch: waiting for a free device slot */
#define COA_QSTAGE_PACK 3        /* launch: parts -> page-locked staging */
#define COA_QSTAGE_ENQUEUE 4     /* launch: H2D copy, kernels and D2H copy enqueued */
#define COA_QSTAGE_DEVICE_WAIT 5 /* completer: blocked on the window's event */
#define COA_QSTAGE_SCATTER 6     /* completer: outputs -> the parts' verdicts */
#define COA_QSTAGE_CALLBACKS 7   /* completer (and helpers): the callbacks */
#define COA_QSTAGE_RESOLVE 8     /* resolver: exact decision of the deferred requests */
#define COA_QSTAGES 9
#define COA_QUEUE_KIND_SIGNATURES 1u
#define COA_QUEUE_KIND_BATCHES 2u
#define COA_QUEUE_KIND_CERTIFICATES 4u
#define COA_QUEUE_KIND_DIGESTS 8u
/* COA_QUEUE_STREAMS=plain|cumask|priority (read at the first launch): plain
 * streams share the process's GPU_MAX_HW_QUEUES hardware queues (HIP's
 * default 4) with every other stream of the process; CU-masked streams (all
 * CUs enabled) get a hardware queue each, whatever GPU_MAX_HW_QUEUES says;
 * priority streams come from the high-priority pool (verify lane) */
#define COA_QUEUE_STREAM_PLAIN 0
#define COA_QUEUE_STREAM_CUMASK 1
#define COA_QUEUE_STREAM_PRIORITY 2
int coa_queue_metrics(coa_queue* q, coa_queue_metrics_t* out);
/* Zeroes the counters, maxima, stage times and the wait histogram (not the
 * slot counts): the next coa_queue_metrics covers only what happens after,
 * e.g. a steady-state interval after a warm-up.  No reference counterpart. */
int coa_queue_metrics_reset(coa_queue* q);
int coa_queue_destroy(coa_queue* q);

#ifdef __cplusplus
}
#endif
#endif /* COA_VERIFY_H */
