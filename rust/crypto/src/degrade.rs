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
//!   * `cpu` (the default) -- the call is answered by the reference's OWN
//!     code on the calling thread: `ed25519_dalek` 1.0.1's `verify_strict` /
//!     `verify_batch` and its `Sha512` re-export, exactly the bodies of
//!     crypto/src/lib.rs:200-219 and the digest sites
//!     (worker/src/processor.rs:38, primary/src/messages.rs:70-84,226-233).
//!     The verdicts are dalek's by construction: the fallback IS the
//!     replaced implementation, which the crate keeps as a dependency for
//!     signing anyway.  Nothing here is the test oracle (oracle/ is test
//!     infrastructure and is never linked into the product).  Each degraded
//!     call is counted (`degraded_calls`) and the first ones are reported on
//!     stderr with the engine's status, so a node running on its CPU is
//!     visible rather than silently slow (~0.03 ms per signature, ~1 ms per
//!     committee-100 certificate on one core).
//!   * `panic` -- the round-4 behaviour: the caller panics with the engine's
//!     message (for deployments that would rather restart a node than run it
//!     at CPU speed).
//!
//! Wiring: `pub mod degrade;` in crypto/src/lib.rs, used by gpu.rs,
//! service.rs and the primary's gpu_certificate.rs.
use crate::{CryptoError, Digest, PublicKey};
use ed25519_dalek as dalek;
use ed25519_dalek::ed25519;
use ed25519_dalek::Digest as _;
use ed25519_dalek::Sha512;
use std::convert::TryInto;
use std::sync::atomic::{AtomicU64, AtomicU8, Ordering};

static DEGRADED: AtomicU64 = AtomicU64::new(0);
/// 0 = not read yet, 1 = cpu, 2 = panic
static POLICY: AtomicU8 = AtomicU8::new(0);
/// Degraded calls reported on stderr before going quiet (the counter keeps
/// counting).
const REPORTED: u64 = 16;

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
/// panics under the `panic` policy, otherwise counts and reports the call,
/// which the caller then answers with the reference's own code.
pub fn engine_failed(rc: i32, msg: &str, what: &str) {
    if panics() {
        panic!("MI355X verification engine failure {} in {}: {}", rc, what, msg);
    }
    let n = DEGRADED.fetch_add(1, Ordering::Relaxed) + 1;
    if n <= REPORTED {
        eprintln!(
            "MI355X verification engine failure {} in {} ({}): answered on the CPU by ed25519-dalek (degraded call #{}{})",
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

/// `Signature::verify` (crypto/src/lib.rs:200-204), the reference's body.
pub fn verify_strict(signature: &[u8; 64], digest: &Digest, public_key: &PublicKey) -> Result<(), CryptoError> {
    let signature = ed25519::signature::Signature::from_bytes(signature)?;
    let key = dalek::PublicKey::from_bytes(&public_key.0)?;
    key.verify_strict(&digest.0, &signature)
}

/// `Signature::verify_batch` (crypto/src/lib.rs:206-219), the reference's
/// body over (key, signature bytes) pairs.
pub fn verify_batch(digest: &Digest, votes: &[(PublicKey, [u8; 64])]) -> Result<(), CryptoError> {
    let mut messages: Vec<&[u8]> = Vec::new();
    let mut signatures: Vec<dalek::Signature> = Vec::new();
    let mut keys: Vec<dalek::PublicKey> = Vec::new();
    for (key, sig) in votes {
        messages.push(&digest.0[..]);
        signatures.push(ed25519::signature::Signature::from_bytes(sig)?);
        keys.push(dalek::PublicKey::from_bytes(&key.0)?);
    }
    dalek::verify_batch(&messages[..], &signatures[..], &keys[..])
}

/// `Digest(Sha512(bytes)[..32])` (worker/src/processor.rs:38).
pub fn sha512_digest(bytes: &[u8]) -> Digest {
    Digest(Sha512::digest(bytes).as_slice()[..32].try_into().unwrap())
}

fn array32(b: &[u8]) -> [u8; 32] {
    b.try_into().expect("32-byte field")
}
fn array64(b: &[u8]) -> [u8; 64] {
    b.try_into().expect("64-byte field")
}

/// The COA_CERT_* bits of `Certificate::verify`'s three crypto checks
/// (primary/src/messages.rs:48-67,189-215), each evaluated on its own as the
/// engine reports them: bit 0 `Header::digest != id` (:70-84), bit 1 the
/// header's `Signature::verify(id, author)` (:64-66), bit 2
/// `Signature::verify_batch(Certificate::digest, votes)` (:214, digest
/// :226-233: id || round LE || origin).  Inputs as the engine takes them:
/// the header's digest input, id, origin, header signature, round and the
/// votes' concatenated 32-byte keys and 64-byte signatures.
pub fn certificate_bits(header_input: &[u8], id: &[u8], origin: &[u8], header_signature: &[u8], round: u64,
                        vote_keys: &[u8], vote_signatures: &[u8]) -> u8 {
    let id = Digest(array32(id));
    let origin = PublicKey(array32(origin));
    let mut bits = 0u8;
    if sha512_digest(header_input) != id {
        bits |= 1;
    }
    if verify_strict(&array64(header_signature), &id, &origin).is_err() {
        bits |= 2;
    }
    let mut hasher = Sha512::new();
    hasher.update(&id.0);
    hasher.update(round.to_le_bytes());
    hasher.update(&origin.0);
    let cert_digest = Digest(hasher.finalize().as_slice()[..32].try_into().unwrap());
    let votes: Vec<(PublicKey, [u8; 64])> = vote_keys
        .chunks_exact(32)
        .zip(vote_signatures.chunks_exact(64))
        .map(|(k, s)| (PublicKey(array32(k)), array64(s)))
        .collect();
    if verify_batch(&cert_digest, &votes).is_err() {
        bits |= 4;
    }
    bits
}
