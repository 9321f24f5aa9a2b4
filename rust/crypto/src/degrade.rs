//! What the drop-in does when the MI355X engine cannot answer at all.
//!
//! The engine already recovers from device faults on its own: a failed shard
//! or queue window is re-run on a rebuilt context, then on every other
//! context of every GPU (`coa_engine_recoveries`, `coa_queue_metrics`'
//! retried / recovered counters).  Only when every attempt failed -- or no
//! GPU was ever found -- does a call return a negative status.  The
//! reference's `Signature::verify` cannot fail for any reason but the
//! signature (crypto/src/lib.rs:200-219), and `Core::run` logs every error
//! and carries on (primary/src/core.rs:390-398), so an engine failure must
//! never become a verdict ("verdicts never depend on device
//! health").
//!
//! Policy, chosen by `COA_ON_ENGINE_FAILURE` (read once per process):
//!   * `cpu` (the default) -- the call is answered by the ENGINE'S OWN CPU
//!     path, `coa_cpu_*` in include/coa_verify.h (csrc/coa_cpu.cpp: the same
//!     dalek 1.0.1 acceptance rules as the GPU kernels, radix-2^51 field
//!     arithmetic and Straus windows on the host's cores, checked against the
//!     golden fixtures and the test oracle by tests/test_cpu_path.py).  It is
//!     neither ed25519-dalek (the replaced implementation) nor the test
//!     oracle (oracle/, never linked into the product).  Each degraded call
//!     is counted (`degraded_calls`) and the first ones are reported on
//!     stderr with the engine's status, so a node running on its CPU is
//!     visible rather than silently slow.
//!   * `panic` -- the caller panics with the engine's message (for
//!     deployments that would rather restart a node than run it at CPU
//!     speed).
//!
//! Wiring: `pub mod degrade;` in crypto/src/lib.rs, used by gpu.rs,
//! service.rs and the primary's gpu_certificate.rs.
use crate::coa_ffi as ffi;
use crate::{CryptoError, Digest, PublicKey};
use std::sync::atomic::{AtomicU64, AtomicU8, Ordering};

static DEGRADED: AtomicU64 = AtomicU64::new(0);
/// 0 = not read yet, 1 = cpu, 2 = panic
static POLICY: AtomicU8 = AtomicU8::new(0);
/// Degraded calls reported on stderr before going quiet (the counter keeps
/// counting).
const REPORTED: u64 = 16;
/// Host threads of the CPU path (0 = min(16, hardware threads)).
const CPU_THREADS: i32 = 0;

fn panics() -> bool {
    let mut p = POLICY.load(Ordering::Relaxed);
    if p == 0 {
        p = match std::env::var("COA_ON_ENGINE_FAILURE") {
            Ok(v) if v == "panic" => 2,
            _ => 1,
        };
        POLICY.store(p, Ordering::Relaxed);
    }
    p == 2
}

/// An engine call of kind `what` returned status `rc` < 0 (message `msg`):
/// panics under the `panic` policy, otherwise counts and reports the call
/// once (a window of many certificates is one call), which the caller then
/// answers with the engine's CPU path.
pub fn engine_failed(rc: i32, msg: &str, what: &str) {
    if panics() {
        panic!("MI355X verification engine failure {} in {}: {}", rc, what, msg);
    }
    let n = DEGRADED.fetch_add(1, Ordering::Relaxed) + 1;
    if n <= REPORTED {
        eprintln!(
            "MI355X verification engine failure {} in {} ({}): answered by the engine's CPU path (degraded call #{}{})",
            rc,
            what,
            msg,
            n,
            if n == REPORTED { "; further ones are counted, not reported" } else { "" }
        );
    }
}

/// Calls answered on the CPU since the process started.
pub fn degraded_calls() -> u64 {
    DEGRADED.load(Ordering::Relaxed)
}

/// The CPU path answers every well-formed call; a negative status here means
/// the arguments themselves were malformed, which no verdict can paper over.
fn cpu_status(rc: i32, what: &str) -> i32 {
    assert!(rc >= 0, "engine CPU path refused {}: status {}", what, rc);
    rc
}

fn result_of(v: i32) -> Result<(), CryptoError> {
    if v == 0 {
        Ok(())
    } else {
        Err(CryptoError::new())
    }
}

/// `Signature::verify` (crypto/src/lib.rs:200-204) on the engine's CPU path.
pub fn cpu_verify(signature: &[u8; 64], digest: &Digest, public_key: &PublicKey) -> Result<(), CryptoError> {
    let rc = unsafe {
        ffi::coa_cpu_ed25519_verify_strict(digest.0.as_ptr(), 32, public_key.0.as_ptr(), signature.as_ptr())
    };
    result_of(cpu_status(rc, "Signature::verify"))
}

/// `Signature::verify_batch` (crypto/src/lib.rs:206-219) on the engine's CPU
/// path, weights from OS entropy (rng_seed 0) as dalek's thread_rng.
pub fn cpu_verify_batch(digest: &Digest, votes: &[(PublicKey, [u8; 64])]) -> Result<(), CryptoError> {
    let (mut pks, mut sigs) = (Vec::with_capacity(32 * votes.len()), Vec::with_capacity(64 * votes.len()));
    for (key, sig) in votes {
        pks.extend_from_slice(&key.0);
        sigs.extend_from_slice(sig);
    }
    let rc = unsafe {
        ffi::coa_cpu_ed25519_verify_batch(digest.0.as_ptr(), pks.as_ptr(), sigs.as_ptr(), votes.len(), 0)
    };
    result_of(cpu_status(rc, "Signature::verify_batch"))
}

/// `Digest(Sha512(bytes)[..32])` (worker/src/processor.rs:38) on the CPU path.
pub fn cpu_digest(bytes: &[u8]) -> Digest {
    let offsets = [0u64, bytes.len() as u64];
    let mut out = [0u8; 64];
    let rc = unsafe { ffi::coa_cpu_sha512_many(bytes.as_ptr(), offsets.as_ptr(), 1, out.as_mut_ptr(), 1) };
    cpu_status(rc, "Digest");
    let mut d = [0u8; 32];
    d.copy_from_slice(&out[..32]);
    Digest(d)
}

/// The COA_CERT_* bits of `Certificate::verify`'s three crypto checks
/// (primary/src/messages.rs:48-67,189-215), each evaluated on its own as the
/// engine reports them: bit 0 `Header::digest != id` (:70-84), bit 1 the
/// header's `Signature::verify(id, author)` (:64-66), bit 2
/// `Signature::verify_batch(Certificate::digest, votes)` (:214, digest
/// :226-233).  Inputs as the engine takes them: the header's digest input,
/// id, origin, header signature, round and the votes' concatenated 32-byte
/// keys and 64-byte signatures.
pub fn cpu_certificate_bits(header_input: &[u8], id: &[u8], origin: &[u8], header_signature: &[u8], round: u64,
                            vote_keys: &[u8], vote_signatures: &[u8]) -> u8 {
    assert!(id.len() == 32 && origin.len() == 32 && header_signature.len() == 64);
    let hoff = [0u64, header_input.len() as u64];
    let voff = [0u64, (vote_keys.len() / 32) as u64];
    let mut status = [0xffu8; 1];
    let rc = unsafe {
        ffi::coa_cpu_certificate_verify_many(header_input.as_ptr(), hoff.as_ptr(), id.as_ptr(), origin.as_ptr(),
                                             header_signature.as_ptr(), &round, vote_keys.as_ptr(),
                                             vote_signatures.as_ptr(), voff.as_ptr(), 1, 0, status.as_mut_ptr(),
                                             CPU_THREADS)
    };
    cpu_status(rc, "Certificate::verify");
    status[0]
}
