//! Raw FFI of the MI355X (gfx950) verification engine: one `extern "C"`
//! declaration per entry point of `include/coa_verify.h`, same names, same
//! argument order and meaning (size_t = usize, uint64_t = u64, void* = *mut
//! c_void).  `tests/test_rust_shim.py` checks this file against the header
//! (every function present, same parameter count and kinds).
//!
//! Verdict convention: 0 = Ok, 1 = Err (the opaque `ed25519::Error`),
//! negative = engine failure (COA_E*).  There is no CPU fallback: without a
//! GPU every call returns COA_ENODEVICE.
#![allow(dead_code)]
use std::os::raw::{c_char, c_int, c_void};

pub const COA_OK: c_int = 0;
pub const COA_REJECT: c_int = 1;
pub const COA_EINVAL: c_int = -1;
pub const COA_ENODEVICE: c_int = -2;
pub const COA_EHIP: c_int = -3;
pub const COA_ENOMEM: c_int = -4;

pub const COA_CERT_BAD_HEADER_ID: c_int = 1;
pub const COA_CERT_BAD_HEADER_SIG: c_int = 2;
pub const COA_CERT_BAD_VOTES: c_int = 4;

pub const COA_MSG_HEADER: i32 = 0;
pub const COA_MSG_VOTE: i32 = 1;
pub const COA_MSG_CERTIFICATE: i32 = 2;
pub const COA_MSG_CERT_REQUEST: i32 = 3;
pub const COA_WIRE_ETRUNC: i32 = -10;
pub const COA_WIRE_EFORMAT: i32 = -11;
pub const COA_WIRE_EKEY: i32 = -12;

/// Opaque aggregation queue (coa_queue_create / coa_queue_destroy).
#[repr(C)]
pub struct CoaQueue {
    _private: [u8; 0],
}

/// coa_queue_metrics_t
#[repr(C)]
#[derive(Default, Debug, Clone, Copy)]
pub struct CoaQueueMetrics {
    pub requests: u64,
    pub windows: u64,
    pub signatures: u64,
    pub batches: u64,
    pub certificates: u64,
    pub digests: u64,
    pub max_window: u64,
    pub max_in_flight: u64,
    pub max_pending: u64,
    pub wait_us_mean: f64,
    pub wait_us_p50: f64,
    pub wait_us_p99: f64,
    pub wait_us_max: f64,
    pub retried_windows: u64,
    pub recovered_windows: u64,
    pub failed_windows: u64,
    pub window_us_max: f64,
    pub window_max_items: u64,
    pub window_max_kinds: u32,
    pub stream_kind: i32,
    pub slot_wait_us_max: f64,
    pub staging_grows: u64,
    pub slots_verify: u32,
    pub slots_digest: u32,
    pub deferred_requests: u64,
    pub resolver_passes: u64,
    pub resolve_us_max: f64,
    /// COA_QSTAGE_* (intake, gather, slot_wait, pack, enqueue, device_wait,
    /// scatter, callbacks, resolve), microseconds summed over windows
    pub stage_us: [f64; 12],
    /// when the slowest window was launched (ms since creation or reset) and
    /// its device wait (µs)
    pub window_max_at_ms: f64,
    pub window_max_device_us: f64,
}

/// void (*coa_verdict_cb)(void* user, int status, const uint8_t* verdicts, size_t n)
pub type CoaVerdictCb = Option<unsafe extern "C" fn(user: *mut c_void, status: c_int, verdicts: *const u8, n: usize)>;

#[link(name = "coa_verify")]
extern "C" {
    // ---------------------------------------------------------- lifecycle
    pub fn coa_init(n_gpus: c_int) -> c_int;
    pub fn coa_init_devices(device_ids: *const c_int, n: c_int) -> c_int;
    pub fn coa_shutdown() -> c_int;
    pub fn coa_device_count() -> c_int;
    pub fn coa_device_ids(ids_out: *mut c_int, cap: c_int) -> c_int;
    pub fn coa_self_test(device: c_int, bad_entries: *mut u64) -> c_int;
    pub fn coa_fe_rows_check_device(device: c_int, d_in: *const u8, n: usize, d_out: *mut u32,
                                    stream: *mut c_void) -> c_int;
    pub fn coa_last_error() -> *const c_char;
    pub fn coa_engine_recoveries(contexts_rebuilt: *mut u64, shards_rerun: *mut u64) -> c_int;
    pub fn coa_version() -> *const c_char;

    // -------------------------------------------------- Signature::verify
    pub fn coa_ed25519_verify_strict(msg: *const u8, pk: *const u8, sig: *const u8) -> c_int;
    pub fn coa_ed25519_verify_strict_many(msgs: *const u8, msg_len: usize, pks: *const u8, sigs: *const u8,
                                          n: usize, verdicts_out: *mut u8) -> c_int;
    pub fn coa_verify_workspace_bytes(n: usize) -> usize;
    pub fn coa_ed25519_verify_strict_many_device(device: c_int, d_msgs: *const u8, msg_len: usize,
                                                 d_pks: *const u8, d_sigs: *const u8, n: usize,
                                                 d_verdicts: *mut u8, workspace: *mut c_void,
                                                 stream: *mut c_void) -> c_int;
    pub fn coa_ed25519_challenge_many_device(device: c_int, d_msgs: *const u8, msg_len: usize, d_pks: *const u8,
                                             d_sigs: *const u8, n: usize, d_k_out: *mut u8,
                                             stream: *mut c_void) -> c_int;
    pub fn coa_ed25519_verify_prehashed_many_device(device: c_int, d_k: *const u8, d_pks: *const u8,
                                                    d_sigs: *const u8, n: usize, d_verdicts: *mut u8,
                                                    workspace: *mut c_void, stream: *mut c_void) -> c_int;

    // -------------------------------------------- Signature::verify_batch
    pub fn coa_ed25519_verify_batch(msg: *const u8, pks: *const u8, sigs: *const u8, n: usize,
                                    rng_seed: u64) -> c_int;
    pub fn coa_ed25519_verify_batch_groups(msgs: *const u8, pks: *const u8, sigs: *const u8,
                                           group_offsets: *const u64, n_groups: usize,
                                           group_verdicts_out: *mut u8, rng_seed: u64) -> c_int;
    pub fn coa_ed25519_verify_batch_groups_z(msgs: *const u8, pks: *const u8, sigs: *const u8,
                                             group_offsets: *const u64, n_groups: usize, zs: *const u8,
                                             group_verdicts_out: *mut u8) -> c_int;
    pub fn coa_verify_batch_workspace_bytes(n: usize) -> usize;
    pub fn coa_ed25519_verify_batch_device(device: c_int, d_msg: *const u8, d_pks: *const u8, d_sigs: *const u8,
                                           n: usize, d_zs: *const u8, rng_seed: u64, d_verdict: *mut u8,
                                           workspace: *mut c_void, workspace_bytes: usize,
                                           stream: *mut c_void) -> c_int;

    // ------------------------------------------------------------- Digest
    pub fn coa_sha512_many(data: *const u8, offsets: *const u64, n: usize, out64: *mut u8) -> c_int;
    pub fn coa_sha512_trunc32_many(data: *const u8, offsets: *const u64, n: usize, out32: *mut u8) -> c_int;
    pub fn coa_sha512_many_device(device: c_int, d_data: *const u8, d_offsets: *const u64, n: usize,
                                  d_out64: *mut u8, stream: *mut c_void) -> c_int;

    // ------------------------------------------ committee key cache (f2)
    pub fn coa_committee_register(pks: *const u8, n: usize) -> c_int;
    pub fn coa_committee_key_flags(flags_out: *mut u32, cap: usize) -> c_int;

    // --------------------------------------- Certificate::verify crypto (f3)
    pub fn coa_certificate_verify_many(header_data: *const u8, header_offsets: *const u64, ids: *const u8,
                                       origins: *const u8, header_sigs: *const u8, rounds: *const u64,
                                       vote_pks: *const u8, vote_sigs: *const u8, vote_offsets: *const u64,
                                       n: usize, rng_seed: u64, status_out: *mut u8) -> c_int;
    pub fn coa_certificate_verify(header_data: *const u8, header_len: usize, id: *const u8, origin: *const u8,
                                  header_sig: *const u8, round: u64, vote_pks: *const u8, vote_sigs: *const u8,
                                  n_votes: usize, rng_seed: u64) -> c_int;
    pub fn coa_certificate_workspace_bytes(n: usize, n_votes: usize) -> usize;
    pub fn coa_certificate_verify_many_device(device: c_int, d_header_data: *const u8,
                                              d_header_offsets: *const u64, d_ids: *const u8,
                                              d_origins: *const u8, d_header_sigs: *const u8,
                                              d_rounds: *const u64, d_vote_pks: *const u8,
                                              d_vote_sigs: *const u8, d_vote_offsets: *const u64, n: usize,
                                              n_votes: usize, d_status: *mut u32, workspace: *mut c_void,
                                              stream: *mut c_void) -> c_int;

    // --------------------------------------------------- wire decode (f4)
    pub fn coa_wire_scan(frames: *const u8, frame_offsets: *const u64, n: usize, kind_out: *mut i32,
                         header_bytes_out: *mut u64, votes_out: *mut u64) -> c_int;
    pub fn coa_wire_decode_certificates(frames: *const u8, frame_offsets: *const u64, n: usize,
                                        header_data: *mut u8, header_offsets: *mut u64, ids: *mut u8,
                                        origins: *mut u8, header_sigs: *mut u8, rounds: *mut u64,
                                        vote_pks: *mut u8, vote_sigs: *mut u8, vote_offsets: *mut u64,
                                        payload_counts: *mut u32) -> c_int;
    pub fn coa_wire_decode_votes(frames: *const u8, frame_offsets: *const u64, n: usize, ids: *mut u8,
                                 rounds: *mut u64, origins: *mut u8, authors: *mut u8, sigs: *mut u8) -> c_int;
    pub fn coa_wire_decode_headers(frames: *const u8, frame_offsets: *const u64, n: usize, header_data: *mut u8,
                                   header_offsets: *mut u64, ids: *mut u8, authors: *mut u8, sigs: *mut u8,
                                   rounds: *mut u64, payload_counts: *mut u32) -> c_int;

    // ----------------------------------------------------------- signing
    pub fn coa_ed25519_public_keys(seeds: *const u8, n: usize, pks_out: *mut u8) -> c_int;
    pub fn coa_ed25519_sign_many(seeds: *const u8, msgs: *const u8, msg_len: usize, n: usize, pks_out: *mut u8,
                                 sigs_out: *mut u8) -> c_int;
    pub fn coa_ed25519_sign_many_device(device: c_int, d_seeds: *const u8, d_msgs: *const u8, msg_len: usize,
                                        n: usize, d_pks_out: *mut u8, d_sigs_out: *mut u8,
                                        stream: *mut c_void) -> c_int;

    // ------------------------------------------ the engine's own CPU path
    // explicit only: degrade.rs calls these after an engine failure
    pub fn coa_cpu_ed25519_verify_strict(msg: *const u8, msg_len: usize, pk: *const u8, sig: *const u8) -> c_int;
    pub fn coa_cpu_ed25519_verify_strict_many(msgs: *const u8, msg_len: usize, pks: *const u8, sigs: *const u8,
                                              n: usize, verdicts_out: *mut u8, nthreads: c_int) -> c_int;
    pub fn coa_cpu_ed25519_verify_batch(msg: *const u8, pks: *const u8, sigs: *const u8, n: usize,
                                        rng_seed: u64) -> c_int;
    pub fn coa_cpu_ed25519_verify_batch_groups_z(msgs: *const u8, pks: *const u8, sigs: *const u8,
                                                 group_offsets: *const u64, n_groups: usize, zs: *const u8,
                                                 group_verdicts_out: *mut u8, nthreads: c_int) -> c_int;
    pub fn coa_cpu_sha512_many(data: *const u8, offsets: *const u64, n: usize, out64: *mut u8,
                               nthreads: c_int) -> c_int;
    pub fn coa_cpu_certificate_verify_many(header_data: *const u8, header_offsets: *const u64, ids: *const u8,
                                           origins: *const u8, header_sigs: *const u8, rounds: *const u64,
                                           vote_pks: *const u8, vote_sigs: *const u8, vote_offsets: *const u64,
                                           n: usize, rng_seed: u64, status_out: *mut u8, nthreads: c_int) -> c_int;
    pub fn coa_cpu_certificate_verify_many_z(header_data: *const u8, header_offsets: *const u64, ids: *const u8,
                                             origins: *const u8, header_sigs: *const u8, rounds: *const u64,
                                             vote_pks: *const u8, vote_sigs: *const u8, vote_offsets: *const u64,
                                             n: usize, zs: *const u8, status_out: *mut u8,
                                             nthreads: c_int) -> c_int;

    // ------------------------------------------------- aggregation queue (f1)
    pub fn coa_queue_create(max_batch: usize, max_delay_us: u32) -> *mut CoaQueue;
    pub fn coa_queue_submit_verify(q: *mut CoaQueue, msg: *const u8, pk: *const u8, sig: *const u8,
                                   cb: CoaVerdictCb, user: *mut c_void) -> c_int;
    pub fn coa_queue_submit_verify_many(q: *mut CoaQueue, msgs: *const u8, pks: *const u8, sigs: *const u8,
                                        n: usize, cb: CoaVerdictCb, user: *mut c_void) -> c_int;
    pub fn coa_queue_submit_batch(q: *mut CoaQueue, msg: *const u8, pks: *const u8, sigs: *const u8, n: usize,
                                  cb: CoaVerdictCb, user: *mut c_void) -> c_int;
    pub fn coa_queue_submit_certificate(q: *mut CoaQueue, header_data: *const u8, header_len: usize,
                                        id: *const u8, origin: *const u8, header_sig: *const u8, round: u64,
                                        vote_pks: *const u8, vote_sigs: *const u8, n_votes: usize,
                                        cb: CoaVerdictCb, user: *mut c_void) -> c_int;
    pub fn coa_queue_submit_certificate_borrowed(q: *mut CoaQueue, header_data: *const u8, header_len: usize,
                                        id: *const u8, origin: *const u8, header_sig: *const u8, round: u64,
                                        vote_pks: *const u8, vote_sigs: *const u8, n_votes: usize,
                                        cb: CoaVerdictCb, user: *mut c_void) -> c_int;
    pub fn coa_queue_submit_digest(q: *mut CoaQueue, data: *const u8, len: usize, cb: CoaVerdictCb,
                                   user: *mut c_void) -> c_int;
    pub fn coa_queue_flush(q: *mut CoaQueue) -> c_int;
    pub fn coa_queue_set_idle_launch(q: *mut CoaQueue, windows_in_flight: u32) -> c_int;
    pub fn coa_queue_stats(q: *mut CoaQueue, launches: *mut u64, items: *mut u64, groups: *mut u64) -> c_int;
    pub fn coa_queue_digest_count(q: *mut CoaQueue, digests: *mut u64) -> c_int;
    pub fn coa_queue_metrics(q: *mut CoaQueue, out: *mut CoaQueueMetrics) -> c_int;
    pub fn coa_queue_metrics_reset(q: *mut CoaQueue) -> c_int;
    pub fn coa_queue_destroy(q: *mut CoaQueue) -> c_int;
}

/// The engine's last error message on this thread (for panics on engine
/// failures).
pub fn last_error() -> String {
    unsafe {
        let p = coa_last_error();
        if p.is_null() {
            String::new()
        } else {
            std::ffi::CStr::from_ptr(p).to_string_lossy().into_owned()
        }
    }
}
