//! The `crypto` crate's hot path on the MI355X engine (`coa_ffi`): the bodies
//! that replace `Signature::verify` and `Signature::verify_batch`
//! (crypto/src/lib.rs:200-219) and the SHA-512 `Digest` of the worker's
//! batches (worker/src/processor.rs:38), plus the committee registration and
//! the batched entry points the aggregation stage uses.
//!
//! Wiring in `crypto/src/lib.rs` (public API unchanged):
//!     mod coa_ffi;            // this crate's src/coa_ffi.rs
//!     pub mod gpu;            // this file
//!     // in impl Signature:
//!     pub fn verify(&self, digest: &Digest, public_key: &PublicKey) -> Result<(), CryptoError> {
//!         gpu::verify(&self.flatten(), digest, public_key)
//!     }
//!     pub fn verify_batch<'a, I>(digest: &Digest, votes: I) -> Result<(), CryptoError>
//!     where I: IntoIterator<Item = &'a (PublicKey, Signature)> {
//!         gpu::verify_batch(digest, votes.into_iter().map(|(k, s)| (k, s.flatten())))
//!     }
//! `ed25519-dalek` stays a dependency for signing (`Signature::new`,
//! `generate_keypair`, `SignatureService`), which is not on the hot path.
//!
//! Also in crypto/src/lib.rs: `pub mod service; pub mod verified;` -- the
//! tokio-side aggregation stage (`service::VerifyService`) and the verdicts
//! it computed ahead of these synchronous calls (`verified`), which
//! `verify` consults first.
use crate::coa_ffi as ffi;
use crate::degrade;
use crate::{CryptoError, Digest, PublicKey};

/// Ok / Err as the engine returned it, or None for an engine failure (no
/// GPU, bad arguments, or a HIP error that persisted after the engine rebuilt
/// the failing context and re-ran the work on every other context,
/// coa_engine_recoveries).  A failure never turns into a verdict: the caller
/// answers with the engine's own CPU path (degrade.rs, coa_cpu_*), or panics
/// under COA_ON_ENGINE_FAILURE=panic.
fn verdict(rc: i32, what: &str) -> Option<Result<(), CryptoError>> {
    match rc {
        ffi::COA_OK => Some(Ok(())),
        ffi::COA_REJECT => Some(Err(CryptoError::new())), // opaque, as ed25519::Error always is
        _ => {
            degrade::engine_failed(rc, &ffi::last_error(), what);
            None
        }
    }
}

/// The 64 bytes R || s of a `Signature` (its private `flatten`,
/// crypto/src/lib.rs:193-198): the primary's callers build engine requests with this
/// instead of a `bincode::serialize` per signature.
pub fn signature_bytes(signature: &crate::Signature) -> [u8; 64] {
    signature.flatten()
}

/// true when the engine answered; false after reporting its failure (the
/// caller then answers with the engine's CPU path, degrade.rs)
fn engine_ok(rc: i32, what: &str) -> bool {
    if rc >= 0 {
        return true;
    }
    degrade::engine_failed(rc, &ffi::last_error(), what);
    false
}

/// Signature::verify (crypto/src/lib.rs:200-204): dalek 1.0.1 verify_strict
/// of the 64-byte signature R || s over the 32-byte digest.  A triple the
/// pre-verification stage already verified (in a coalesced launch; Ok or
/// Err, both exact) is answered from `verified`; any other takes the
/// engine's single-signature latency kernel on an idle device context.
pub fn verify(signature: &[u8; 64], digest: &Digest, public_key: &PublicKey) -> Result<(), CryptoError> {
    if let Some(ok) = crate::verified::take_signature(digest, public_key, signature) {
        return if ok { Ok(()) } else { Err(CryptoError::new()) };
    }
    let rc = unsafe { ffi::coa_ed25519_verify_strict(digest.0.as_ptr(), public_key.0.as_ptr(), signature.as_ptr()) };
    verdict(rc, "Signature::verify").unwrap_or_else(|| degrade::cpu_verify(signature, digest, public_key))
}

/// Signature::verify_batch (crypto/src/lib.rs:206-219): dalek 1.0.1
/// verify_batch over votes that all sign `digest` (random linear
/// combination, weights from OS entropy per call as dalek's thread_rng).
pub fn verify_batch<'a, I>(digest: &Digest, votes: I) -> Result<(), CryptoError>
where
    I: IntoIterator<Item = (&'a PublicKey, [u8; 64])>,
{
    let votes: Vec<(PublicKey, [u8; 64])> = votes.into_iter().map(|(k, s)| (*k, s)).collect();
    let (mut pks, mut sigs) = (Vec::with_capacity(32 * votes.len()), Vec::with_capacity(64 * votes.len()));
    for (key, sig) in &votes {
        pks.extend_from_slice(&key.0);
        sigs.extend_from_slice(sig);
    }
    let rc = unsafe { ffi::coa_ed25519_verify_batch(digest.0.as_ptr(), pks.as_ptr(), sigs.as_ptr(), votes.len(), 0) };
    verdict(rc, "Signature::verify_batch").unwrap_or_else(|| degrade::cpu_verify_batch(digest, &votes))
}

/// Digest(Sha512(bytes)[..32]) of ONE message on the device.  One 508 KB
/// worker batch per launch is a serial chain of 3,970 compressions (~14 ms,
/// against ~1 ms on a CPU core): the worker's `Processor` must not call this
/// per batch -- it streams its batches through `service::VerifyService::
/// digest` instead (rust/worker/src/processor.rs), whose windows hash many
/// batches per launch.
pub fn sha512_digest(bytes: &[u8]) -> Digest {
    let offsets = [0u64, bytes.len() as u64];
    let mut out = [0u8; 32];
    if !engine_ok(unsafe { ffi::coa_sha512_trunc32_many(bytes.as_ptr(), offsets.as_ptr(), 1, out.as_mut_ptr()) },
                  "Sha512 digest") {
        return degrade::cpu_digest(bytes);
    }
    Digest(out)
}

/// Digests of many messages in one launch (the worker's coalescing path).
pub fn sha512_digests(messages: &[&[u8]]) -> Vec<Digest> {
    let mut data = Vec::new();
    let mut offsets = Vec::with_capacity(messages.len() + 1);
    offsets.push(0u64);
    for m in messages {
        data.extend_from_slice(m);
        offsets.push(data.len() as u64);
    }
    let mut out = vec![0u8; 32 * messages.len()];
    if !engine_ok(unsafe {
        ffi::coa_sha512_trunc32_many(data.as_ptr(), offsets.as_ptr(), messages.len(), out.as_mut_ptr())
    }, "Sha512 digests") {
        return messages.iter().map(|m| degrade::cpu_digest(m)).collect();
    }
    out.chunks_exact(32)
        .map(|c| {
            let mut d = [0u8; 32];
            d.copy_from_slice(c);
            Digest(d)
        })
        .collect()
}

/// Registers the committee's keys in the engine's key cache (once after
/// `Committee::import` in node/src/main.rs, and on committee change).  Speed
/// only: verdicts never depend on it.  Returns the number of distinct keys.
pub fn register_committee<'a, I>(keys: I) -> usize
where
    I: IntoIterator<Item = &'a PublicKey>,
{
    let flat: Vec<u8> = keys.into_iter().flat_map(|k| k.0.iter().copied()).collect();
    let rc = unsafe { ffi::coa_committee_register(flat.as_ptr(), flat.len() / 32) };
    // speed only: without a key cache every call still answers exactly
    if engine_ok(rc, "coa_committee_register") { rc as usize } else { 0 }
}

/// Many independent (digest, key, signature) triples in one launch (the
/// aggregation stage in front of Core): one Ok/Err per triple.
pub fn verify_many(items: &[(Digest, PublicKey, [u8; 64])]) -> Vec<Result<(), CryptoError>> {
    let n = items.len();
    let (mut msgs, mut pks, mut sigs) = (Vec::with_capacity(32 * n), Vec::with_capacity(32 * n), Vec::with_capacity(64 * n));
    for (d, k, s) in items {
        msgs.extend_from_slice(&d.0);
        pks.extend_from_slice(&k.0);
        sigs.extend_from_slice(s);
    }
    let mut out = vec![1u8; n];
    if !engine_ok(unsafe {
        ffi::coa_ed25519_verify_strict_many(msgs.as_ptr(), 32, pks.as_ptr(), sigs.as_ptr(), n, out.as_mut_ptr())
    }, "Signature::verify (many)") {
        return items.iter().map(|(d, k, s)| degrade::cpu_verify(s, d, k)).collect();
    }
    out.into_iter().map(|v| if v == 0 { Ok(()) } else { Err(CryptoError::new()) }).collect()
}

/// Many certificates' vote batches in one launch: one verify_batch verdict
/// per group (certificate), votes concatenated, group g = votes of
/// certificate g over digests[g].
pub fn verify_batch_groups(digests: &[Digest], groups: &[Vec<(PublicKey, [u8; 64])>]) -> Vec<Result<(), CryptoError>> {
    assert_eq!(digests.len(), groups.len());
    let mut msgs = Vec::with_capacity(32 * digests.len());
    let (mut pks, mut sigs) = (Vec::new(), Vec::new());
    let mut offsets = Vec::with_capacity(groups.len() + 1);
    offsets.push(0u64);
    for (d, g) in digests.iter().zip(groups) {
        msgs.extend_from_slice(&d.0);
        for (k, s) in g {
            pks.extend_from_slice(&k.0);
            sigs.extend_from_slice(s);
        }
        offsets.push((pks.len() / 32) as u64);
    }
    let mut out = vec![1u8; groups.len()];
    if !engine_ok(unsafe {
        ffi::coa_ed25519_verify_batch_groups(msgs.as_ptr(), pks.as_ptr(), sigs.as_ptr(), offsets.as_ptr(),
                                             groups.len(), out.as_mut_ptr(), 0)
    }, "Signature::verify_batch (groups)") {
        return digests.iter().zip(groups).map(|(d, g)| degrade::cpu_verify_batch(d, g)).collect();
    }
    out.into_iter().map(|v| if v == 0 { Ok(()) } else { Err(CryptoError::new()) }).collect()
}
