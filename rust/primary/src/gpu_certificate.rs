//! `Certificate::verify` (primary/src/messages.rs:189-215) with its crypto in
//! ONE engine call (`coa_certificate_verify`: Header::digest == id, the
//! header's Signature::verify, Certificate::digest and the votes'
//! verify_batch, fused on the device over the registered committee's key
//! combs), the non-crypto checks in the reference's order.  The crypto bits
//! are pure functions of the certificate's bytes, so reading them up front and
//! consuming them in the reference's order returns exactly the reference's
//! DagError.
//!
//! Wiring in `primary/src/messages.rs`:
//!     #[path = "gpu_certificate.rs"] mod gpu_certificate;
//!     impl Certificate {
//!         pub fn verify(&self, committee: &Committee) -> DagResult<()> {
//!             gpu_certificate::verify(self, committee)
//!         }
//!     }
//! and in node/src/main.rs, once after Committee::import:
//!     crypto::gpu::register_committee(committee.authorities.keys());
//! `primary/Cargo.toml` needs nothing new (crypto is already a dependency;
//! the FFI lives in crypto's `coa_ffi`, re-exported below).
//!
//! A certificate the pre-verification stage (pre_verify.rs) already ran
//! through the engine in a coalesced launch is answered from
//! `crypto::verified` (keyed by every byte of its crypto input), so `Core`'s
//! one-at-a-time call costs a lookup instead of a launch.
use crate::error::{DagError, DagResult};
use crate::messages::{Certificate, Header};
use config::Committee;
use crypto::gpu::signature_bytes;
use crypto::service::CertificateCrypto;
use crypto::{CryptoError, PublicKey};
use std::collections::HashSet;
use std::os::raw::c_int;

extern "C" {
    // include/coa_verify.h; the symbols come from libcoa_verify.so, which the
    // crypto crate's build.rs links
    fn coa_certificate_verify(header_data: *const u8, header_len: usize, id: *const u8, origin: *const u8,
                              header_sig: *const u8, round: u64, vote_pks: *const u8, vote_sigs: *const u8,
                              n_votes: usize, rng_seed: u64) -> c_int;
    fn coa_certificate_verify_many(header_data: *const u8, header_offsets: *const u64, ids: *const u8,
                                   origins: *const u8, header_sigs: *const u8, rounds: *const u64,
                                   vote_pks: *const u8, vote_sigs: *const u8, vote_offsets: *const u64,
                                   n: usize, rng_seed: u64, status_out: *mut u8) -> c_int;
    fn coa_cpu_certificate_verify_many(header_data: *const u8, header_offsets: *const u64, ids: *const u8,
                                       origins: *const u8, header_sigs: *const u8, rounds: *const u64,
                                       vote_pks: *const u8, vote_sigs: *const u8, vote_offsets: *const u64,
                                       n: usize, rng_seed: u64, status_out: *mut u8, nthreads: c_int) -> c_int;
    fn coa_last_error() -> *const std::os::raw::c_char;
}

const BAD_HEADER_ID: c_int = 1;
const BAD_HEADER_SIG: c_int = 2;
const BAD_VOTES: c_int = 4;

/// An engine failure (every context failed, or no GPU): reported once per
/// call (or a panic under COA_ON_ENGINE_FAILURE=panic); the caller then takes
/// the certificates' crypto bits from the engine's own CPU path
/// (coa_cpu_certificate_verify_many, crypto/src/degrade.rs), so the DagError
/// is still the reference's.
fn engine_failure(rc: c_int) {
    let msg = unsafe { std::ffi::CStr::from_ptr(coa_last_error()) }.to_string_lossy().into_owned();
    crypto::degrade::engine_failed(rc, &msg, "Certificate::verify");
}

/// The COA_CERT_* bits of one certificate on the engine's CPU path.
fn cpu_bits(c: &CertificateCrypto) -> c_int {
    crypto::degrade::cpu_certificate_bits(c.header_input(), c.id(), c.origin(), c.header_signature(), c.round(),
                                          c.vote_keys(), c.vote_signatures()) as c_int
}

/// Length of the bytes Header::digest hashes (primary/src/messages.rs:70-84).
pub fn header_digest_len(h: &Header) -> usize {
    32 + 8 + 36 * h.payload.len() + 32 * h.parents.len()
}

/// Appends the bytes Header::digest hashes (primary/src/messages.rs:70-84):
/// author || round (u64 LE) || (payload digest || worker id (u32 LE))* in the
/// BTreeMap's key order || parent digests in the BTreeSet's order.
pub fn write_header_digest_input(h: &Header, out: &mut Vec<u8>) {
    out.extend_from_slice(&h.author.0);
    out.extend_from_slice(&h.round.to_le_bytes());
    for (digest, worker_id) in &h.payload {
        out.extend_from_slice(&digest.0);
        out.extend_from_slice(&worker_id.to_le_bytes());
    }
    for parent in &h.parents {
        out.extend_from_slice(&parent.0);
    }
}

/// The crypto input of Certificate::verify in the engine's terms (the
/// request `VerifyService::certificate` and `coa_certificate_verify` take),
/// built once in one buffer of its exact size: the signatures' bytes come
/// from `crypto::gpu::signature_bytes` (no `bincode::serialize` per vote),
/// and the buffer is also the `verified` cache key (no second copy).
pub(crate) fn certificate_crypto(cert: &Certificate) -> CertificateCrypto {
    let h = &cert.header;
    CertificateCrypto::new(header_digest_len(h), |out| write_header_digest_input(h, out), &h.id, &h.author,
                           &h.signature, h.round, &cert.votes)
}

/// The checks of Certificate::verify in the reference's order, the crypto
/// ones read from the engine's status bits.
fn checks_in_order(cert: &Certificate, committee: &Committee, st: c_int) -> DagResult<()> {
    let h = &cert.header;
    // Header::verify (:48-67)
    ensure!(st & BAD_HEADER_ID == 0, DagError::InvalidHeaderId);
    ensure!(committee.stake(&h.author) > 0, DagError::UnknownAuthority(h.author));
    for worker_id in h.payload.values() {
        committee
            .worker(&h.author, worker_id)
            .map_err(|_| DagError::MalformedHeader(h.id.clone()))?;
    }
    ensure!(st & BAD_HEADER_SIG == 0, DagError::InvalidSignature(CryptoError::new()));
    // quorum (:196-211)
    let mut weight = 0;
    let mut used: HashSet<PublicKey> = HashSet::new();
    for (name, _) in cert.votes.iter() {
        ensure!(!used.contains(name), DagError::AuthorityReuse(*name));
        let voting_rights = committee.stake(name);
        ensure!(voting_rights > 0, DagError::UnknownAuthority(*name));
        used.insert(*name);
        weight += voting_rights;
    }
    ensure!(weight >= committee.quorum_threshold(), DagError::CertificateRequiresQuorum);
    // verify_batch (:214)
    ensure!(st & BAD_VOTES == 0, DagError::InvalidSignature(CryptoError::new()));
    Ok(())
}

/// Certificate::verify, one certificate: the bits the pre-verification
/// stage computed for exactly these bytes, or the engine's latency path (one
/// launch with the certificate in its arguments, on an idle device context).
pub fn verify(cert: &Certificate, committee: &Committee) -> DagResult<()> {
    // Genesis certificates are always valid (:191-193).
    if Certificate::genesis(committee).contains(cert) {
        return Ok(());
    }
    let c = certificate_crypto(cert);
    if let Some(bits) = crypto::verified::take_certificate(c.key_bytes()) {
        return checks_in_order(cert, committee, bits as c_int);
    }
    let st = unsafe {
        coa_certificate_verify(c.header_input().as_ptr(), c.header_input().len(), c.id().as_ptr(),
                               c.origin().as_ptr(), c.header_signature().as_ptr(), c.round(),
                               c.vote_keys().as_ptr(), c.vote_signatures().as_ptr(), c.n_votes(), 0)
    };
    let st = if st < 0 {
        engine_failure(st);
        cpu_bits(&c)
    } else {
        st
    };
    checks_in_order(cert, committee, st)
}

/// Certificate::verify for a window of certificates (the aggregation stage):
/// the crypto of all of them in one coa_certificate_verify_many call, then
/// each certificate's checks in the reference's order.
pub fn verify_many(certs: &[&Certificate], committee: &Committee) -> Vec<DagResult<()>> {
    let genesis = Certificate::genesis(committee);
    let todo: Vec<usize> = (0..certs.len()).filter(|&i| !genesis.contains(certs[i])).collect();
    let n = todo.len();
    let mut hdata = Vec::new();
    let mut hoff = vec![0u64];
    let (mut ids, mut origins, mut hsigs) = (Vec::with_capacity(32 * n), Vec::with_capacity(32 * n), Vec::with_capacity(64 * n));
    let mut rounds = Vec::with_capacity(n);
    let (mut vpks, mut vsigs) = (Vec::new(), Vec::new());
    let mut voff = vec![0u64];
    for &i in &todo {
        let h = &certs[i].header;
        write_header_digest_input(h, &mut hdata);
        hoff.push(hdata.len() as u64);
        ids.extend_from_slice(&h.id.0);
        origins.extend_from_slice(&h.author.0);
        hsigs.extend_from_slice(&signature_bytes(&h.signature));
        rounds.push(h.round);
        for (name, sig) in &certs[i].votes {
            vpks.extend_from_slice(&name.0);
            vsigs.extend_from_slice(&signature_bytes(sig));
        }
        voff.push((vpks.len() / 32) as u64);
    }
    let mut status = vec![0u8; n];
    if n > 0 {
        let rc = unsafe {
            coa_certificate_verify_many(hdata.as_ptr(), hoff.as_ptr(), ids.as_ptr(), origins.as_ptr(),
                                        hsigs.as_ptr(), rounds.as_ptr(), vpks.as_ptr(), vsigs.as_ptr(),
                                        voff.as_ptr(), n, 0, status.as_mut_ptr())
        };
        if rc < 0 {
            // the whole window answered by the engine's CPU path, one call
            engine_failure(rc);
            let rc = unsafe {
                coa_cpu_certificate_verify_many(hdata.as_ptr(), hoff.as_ptr(), ids.as_ptr(), origins.as_ptr(),
                                                hsigs.as_ptr(), rounds.as_ptr(), vpks.as_ptr(), vsigs.as_ptr(),
                                                voff.as_ptr(), n, 0, status.as_mut_ptr(), 0)
            };
            assert!(rc >= 0, "engine CPU path refused Certificate::verify: status {}", rc);
        }
    }
    let mut out: Vec<DagResult<()>> = (0..certs.len()).map(|_| Ok(())).collect();
    for (j, &i) in todo.iter().enumerate() {
        out[i] = checks_in_order(certs[i], committee, status[j] as c_int);
    }
    out
}
