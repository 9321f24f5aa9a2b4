//! The tokio-side aggregation stage over the engine's native queue
//! (`coa_queue_*`, include/coa_verify.h): `VerifyService`, modelled on the
//! reference's `SignatureService` (crypto/src/lib.rs:222-250) -- an mpsc
//! request channel in, a `oneshot` reply per request.  Where
//! `SignatureService` signs one digest per request, this service hands every
//! request it has received to the engine's queue, which coalesces the
//! requests of all tasks into a few large launches:
//!
//!   * `Signature::verify` triples (Header::verify, Vote::verify,
//!     primary/src/messages.rs:64-66,139-141): whatever the service task
//!     drains from its channel at once goes to the queue as ONE
//!     `coa_queue_submit_verify_many` request whose callback fans the
//!     verdicts out to the requests' oneshot senders;
//!   * vote batches (`Signature::verify_batch`, :206-219), whole certificates
//!     (the fused `Certificate::verify` crypto, messages.rs:189-215) and
//!     worker batch digests (worker/src/processor.rs:38) go one request each.
//!
//! The engine answers on its completion thread through the `extern "C"`
//! callbacks below; each one takes back the boxed sender(s) it was given and
//! completes them.  `oneshot::Sender::send` does not block and needs no
//! runtime, so the callbacks never touch tokio's threads.  A callback never
//! panics (that would unwind across the FFI boundary): an engine failure --
//! reported only after the queue re-ran the window on every device context
//! (coa_queue_metrics' retried/recovered/failed counters) -- travels to the
//! awaiting task as `Err(status)` with the request's inputs handed back, and
//! the task answers it there with the reference's own code (degrade.rs:
//! ed25519-dalek's verify_strict / verify_batch and its Sha512, so the
//! verdict is the reference's), or panics under COA_ON_ENGINE_FAILURE=panic,
//! as the synchronous calls in `gpu.rs` do.
//!
//! Wiring (crypto/src/lib.rs): `pub mod service;`.  One service per process,
//! created once the committee is registered (node/src/main.rs):
//!     let verifier = crypto::service::VerifyService::new(65_536, 500);
use crate::coa_ffi as ffi;
use crate::degrade;
use crate::{CryptoError, Digest, PublicKey};
use std::os::raw::{c_int, c_void};
use tokio::sync::mpsc::{channel, Receiver, Sender};
use tokio::sync::oneshot;

/// A verdict as the crate reports it, or the engine's failure status.
type Verdict = Result<Result<(), CryptoError>, c_int>;

/// The crypto of one `Certificate::verify` in the engine's terms (the
/// `primary` crate builds it: rust/primary/src/gpu_certificate.rs), held in
/// ONE buffer that is also its `verified` cache key -- every byte the
/// verdict depends on, length-framed:
///
///   header_len u64 | header input | id | origin | header signature R || s |
///   round u64 | n_votes u64 | n_votes x key (32) | n_votes x signature (64)
///
/// Built once per certificate with its exact size (no per-vote
/// serialization, no second copy for the key): the queue copies the fields
/// at submission, and the buffer then becomes the cache key as it is.
pub struct CertificateCrypto {
    bytes: Vec<u8>,
    header_len: usize,
    n_votes: usize,
}

impl CertificateCrypto {
    /// `write_header_input` appends the `header_len` bytes `Header::digest`
    /// hashes (primary/src/messages.rs:70-84); `votes` are the certificate's
    /// (key, signature) pairs in order.
    pub fn new<F: FnOnce(&mut Vec<u8>)>(header_len: usize, write_header_input: F, id: &Digest, origin: &PublicKey,
                                        header_signature: &crate::Signature, round: u64,
                                        votes: &[(PublicKey, crate::Signature)]) -> Self {
        let n_votes = votes.len();
        let mut bytes = Vec::with_capacity(8 + header_len + 32 + 32 + 64 + 8 + 8 + 96 * n_votes);
        bytes.extend_from_slice(&(header_len as u64).to_le_bytes());
        write_header_input(&mut bytes);
        assert_eq!(bytes.len(), 8 + header_len, "header input of the announced length");
        bytes.extend_from_slice(&id.0);
        bytes.extend_from_slice(&origin.0);
        bytes.extend_from_slice(&crate::gpu::signature_bytes(header_signature));
        bytes.extend_from_slice(&round.to_le_bytes());
        bytes.extend_from_slice(&(n_votes as u64).to_le_bytes());
        for (key, _) in votes {
            bytes.extend_from_slice(&key.0);
        }
        for (_, signature) in votes {
            bytes.extend_from_slice(&crate::gpu::signature_bytes(signature));
        }
        Self { bytes, header_len, n_votes }
    }

    fn at(&self, field: usize) -> usize {
        // offsets of: header input, id, origin, header signature, round, votes
        let h = 8 + self.header_len;
        [8, h, h + 32, h + 64, h + 128, h + 144][field]
    }
    pub fn header_input(&self) -> &[u8] {
        &self.bytes[8..8 + self.header_len]
    }
    pub fn id(&self) -> &[u8] {
        &self.bytes[self.at(1)..self.at(1) + 32]
    }
    pub fn origin(&self) -> &[u8] {
        &self.bytes[self.at(2)..self.at(2) + 32]
    }
    pub fn header_signature(&self) -> &[u8] {
        &self.bytes[self.at(3)..self.at(3) + 64]
    }
    pub fn round(&self) -> u64 {
        let mut r = [0u8; 8];
        r.copy_from_slice(&self.bytes[self.at(4)..self.at(4) + 8]);
        u64::from_le_bytes(r)
    }
    pub fn n_votes(&self) -> usize {
        self.n_votes
    }
    /// the votes' 32-byte keys, concatenated
    pub fn vote_keys(&self) -> &[u8] {
        &self.bytes[self.at(5)..self.at(5) + 32 * self.n_votes]
    }
    /// the votes' 64-byte signatures, concatenated
    pub fn vote_signatures(&self) -> &[u8] {
        let v = self.at(5) + 32 * self.n_votes;
        &self.bytes[v..v + 64 * self.n_votes]
    }
    /// Every byte the certificate's crypto verdict depends on (the key of
    /// `verified::take_certificate`).
    pub fn key_bytes(&self) -> &[u8] {
        &self.bytes
    }
    /// The same bytes, moved out (the key of `verified::remember_certificate`).
    pub fn into_key(self) -> Vec<u8> {
        self.bytes
    }
}

/// A worker batch on its way through the engine, handed back with its digest
/// (the batch is then stored, worker/src/processor.rs:41) -- or with the
/// engine's failure status, for the CPU answer (degrade.rs).
type DigestReply = Result<(Digest, Vec<u8>), (c_int, Vec<u8>)>;

/// A certificate's COA_CERT_* bits, with its crypto handed back (it becomes
/// the `verified` key without a copy) -- or with the engine's failure status.
type CertificateReply = Result<(u8, CertificateCrypto), (c_int, CertificateCrypto)>;

/// A vote batch's verdict -- or the engine's failure status with the votes
/// handed back (for the CPU answer: no copy kept on the success path).
type BatchReply = Result<Result<(), CryptoError>, (c_int, Vec<(PublicKey, [u8; 64])>)>;

enum Request {
    Verify(Digest, PublicKey, [u8; 64], oneshot::Sender<Verdict>),
    Batch(Digest, Vec<(PublicKey, [u8; 64])>, oneshot::Sender<BatchReply>),
    Certificate(CertificateCrypto, oneshot::Sender<CertificateReply>),
    Digest(Vec<u8>, oneshot::Sender<DigestReply>),
}

/// The engine queue, shared by the service task and the callbacks.  The C
/// queue is thread-safe (per-thread intake shards, its own threads).
struct Queue(*mut ffi::CoaQueue);
unsafe impl Send for Queue {}
unsafe impl Sync for Queue {}

/// Most requests the service task drains from its channel per turn.
const DRAIN: usize = 4096;

#[derive(Clone)]
pub struct VerifyService {
    channel: Sender<Request>,
}

impl VerifyService {
    /// `max_batch`: signatures per GPU launch window (the queue closes a
    /// window when this many are pending); `max_delay_us`: the longest a
    /// request waits for its window to close.
    ///
    /// The queue also launches a window at once while no window is in flight
    /// (`coa_queue_set_idle_launch(q, 1)`): a request reaching an idle engine
    /// does not wait out `max_delay_us`, and under load requests still
    /// coalesce behind the windows in flight (committee-100 round mix p50
    /// 0.31-0.39 ms with the deadline alone, 0.07-0.26 ms with it).
    /// `COA_SERVICE_IDLE_LAUNCH=0` keeps the deadline policy alone.
    pub fn new(max_batch: usize, max_delay_us: u32) -> Self {
        let queue = unsafe { ffi::coa_queue_create(max_batch, max_delay_us) };
        assert!(!queue.is_null(), "MI355X verification engine: coa_queue_create failed: {}", ffi::last_error());
        // windows in flight below which a window launches at once: 0..=64, as
        // coa_queue_create clamps COA_QUEUE_IDLE_LAUNCH (a larger value is
        // taken as 64, never a failed assertion at node start)
        let idle: u32 =
            std::env::var("COA_SERVICE_IDLE_LAUNCH").ok().and_then(|v| v.parse().ok()).unwrap_or(1u32).min(64);
        let rc = unsafe { ffi::coa_queue_set_idle_launch(queue, idle) };
        assert_eq!(rc, ffi::COA_OK, "MI355X verification engine: coa_queue_set_idle_launch({}) failed", idle);
        let queue = Queue(queue);
        let (tx, rx): (Sender<Request>, Receiver<Request>) = channel(DRAIN);
        tokio::spawn(Self::run(queue, rx));
        Self { channel: tx }
    }

    async fn run(queue: Queue, mut rx: Receiver<Request>) {
        while let Some(first) = rx.recv().await {
            let mut window = vec![first];
            while window.len() < DRAIN {
                match rx.try_recv() {
                    Ok(request) => window.push(request),
                    Err(_) => break,
                }
            }
            submit_window(&queue, window);
        }
        // every handle dropped: answer what is in flight, then free the queue
        // (both block, so off the async workers)
        let _ = tokio::task::spawn_blocking(move || unsafe {
            ffi::coa_queue_flush(queue.0);
            ffi::coa_queue_destroy(queue.0);
        })
        .await;
    }

    async fn send(&self, request: Request) {
        if let Err(e) = self.channel.send(request).await {
            panic!("Failed to send request to the Verify Service: {}", e);
        }
    }

    /// `Signature::verify(digest, key)` (crypto/src/lib.rs:200-204) through
    /// the queue: coalesced with every other pending request.
    pub async fn verify(&self, digest: &Digest, key: &PublicKey, signature: [u8; 64]) -> Result<(), CryptoError> {
        let (sender, receiver) = oneshot::channel();
        self.send(Request::Verify(digest.clone(), *key, signature, sender)).await;
        match receiver.await.expect("Failed to receive verdict from Verify Service") {
            Ok(verdict) => verdict,
            Err(status) => {
                degrade::engine_failed(status, "every context failed", "VerifyService::verify");
                degrade::cpu_verify(&signature, digest, key)
            }
        }
    }

    /// `Signature::verify_batch(digest, votes)` (crypto/src/lib.rs:206-219).
    pub async fn verify_batch(&self, digest: &Digest, votes: Vec<(PublicKey, [u8; 64])>) -> Result<(), CryptoError> {
        let (sender, receiver) = oneshot::channel();
        self.send(Request::Batch(digest.clone(), votes, sender)).await;
        match receiver.await.expect("Failed to receive verdict from Verify Service") {
            Ok(verdict) => verdict,
            Err((status, votes)) => {
                degrade::engine_failed(status, "every context failed", "VerifyService::verify_batch");
                degrade::cpu_verify_batch(digest, &votes)
            }
        }
    }

    /// The crypto of `Certificate::verify` (primary/src/messages.rs:189-215):
    /// the COA_CERT_* bits (0 = every crypto check Ok), and the request
    /// handed back.
    pub async fn certificate(&self, crypto: CertificateCrypto) -> (u8, CertificateCrypto) {
        let (sender, receiver) = oneshot::channel();
        self.send(Request::Certificate(crypto, sender)).await;
        match receiver.await.expect("Failed to receive status from Verify Service") {
            Ok(reply) => reply,
            Err((status, c)) => {
                degrade::engine_failed(status, "every context failed", "VerifyService::certificate");
                let bits = degrade::cpu_certificate_bits(c.header_input(), c.id(), c.origin(),
                                                         c.header_signature(), c.round(), c.vote_keys(),
                                                         c.vote_signatures());
                (bits, c)
            }
        }
    }

    /// `Digest(Sha512(bytes)[..32])` (worker/src/processor.rs:38), with the
    /// bytes handed back (the queue copies them at submission; no clone).
    pub async fn digest(&self, bytes: Vec<u8>) -> (Digest, Vec<u8>) {
        let (sender, receiver) = oneshot::channel();
        self.send(Request::Digest(bytes, sender)).await;
        match receiver.await.expect("Failed to receive digest from Verify Service") {
            Ok(reply) => reply,
            Err((status, bytes)) => {
                degrade::engine_failed(status, "every context failed", "VerifyService::digest");
                (degrade::cpu_digest(&bytes), bytes)
            }
        }
    }
}

fn verdict_of(byte: u8) -> Result<(), CryptoError> {
    if byte == 0 {
        Ok(())
    } else {
        Err(CryptoError::new())
    }
}

/// One drained window of requests into the engine queue.
fn submit_window(queue: &Queue, window: Vec<Request>) {
    let mut senders: Vec<oneshot::Sender<Verdict>> = Vec::new();
    let (mut msgs, mut keys, mut sigs) = (Vec::new(), Vec::new(), Vec::new());
    for request in window {
        match request {
            Request::Verify(digest, key, signature, sender) => {
                msgs.extend_from_slice(&digest.0);
                keys.extend_from_slice(&key.0);
                sigs.extend_from_slice(&signature);
                senders.push(sender);
            }
            Request::Batch(digest, votes, sender) => submit_batch(queue, &digest, votes, sender),
            Request::Certificate(crypto, sender) => submit_certificate(queue, crypto, sender),
            Request::Digest(bytes, sender) => submit_digest(queue, bytes, sender),
        }
    }
    if senders.is_empty() {
        return;
    }
    let n = senders.len();
    let user = Box::into_raw(Box::new(senders)) as *mut c_void;
    let rc = unsafe {
        ffi::coa_queue_submit_verify_many(queue.0, msgs.as_ptr(), keys.as_ptr(), sigs.as_ptr(), n,
                                          Some(on_verdicts), user)
    };
    if rc != ffi::COA_OK {
        // not queued: the callback will never run, so answer here
        let senders = unsafe { Box::from_raw(user as *mut Vec<oneshot::Sender<Verdict>>) };
        for sender in *senders {
            let _ = sender.send(Err(rc));
        }
    }
}

fn submit_batch(queue: &Queue, digest: &Digest, votes: Vec<(PublicKey, [u8; 64])>,
                sender: oneshot::Sender<BatchReply>) {
    let (mut keys, mut sigs) = (Vec::with_capacity(32 * votes.len()), Vec::with_capacity(64 * votes.len()));
    for (key, signature) in &votes {
        keys.extend_from_slice(&key.0);
        sigs.extend_from_slice(signature);
    }
    let n = votes.len();
    // the votes ride along with the sender: handed back only on a failure
    let user = Box::into_raw(Box::new((sender, votes))) as *mut c_void;
    let rc = unsafe {
        ffi::coa_queue_submit_batch(queue.0, digest.0.as_ptr(), keys.as_ptr(), sigs.as_ptr(), n, Some(on_batch),
                                    user)
    };
    if rc != ffi::COA_OK {
        let pair = unsafe { Box::from_raw(user as *mut (oneshot::Sender<BatchReply>, Vec<(PublicKey, [u8; 64])>)) };
        let (sender, votes) = *pair;
        let _ = sender.send(Err((rc, votes)));
    }
}

fn submit_certificate(queue: &Queue, crypto: CertificateCrypto, sender: oneshot::Sender<CertificateReply>) {
    // the request rides along with the sender and comes back with the bits:
    // its buffer lives (boxed, never moved: the Vec's heap block stays put)
    // until the callback has run, so the queue reads it in place
    // (coa_queue_submit_certificate_borrowed: no intake copy; the window's
    // launch packs it straight into the device staging)
    let user = Box::into_raw(Box::new((sender, crypto))) as *mut c_void;
    let c = unsafe { &(*(user as *const (oneshot::Sender<CertificateReply>, CertificateCrypto))).1 };
    let rc = unsafe {
        ffi::coa_queue_submit_certificate_borrowed(queue.0, c.header_input().as_ptr(), c.header_input().len(),
                                          c.id().as_ptr(), c.origin().as_ptr(), c.header_signature().as_ptr(),
                                          c.round(), c.vote_keys().as_ptr(), c.vote_signatures().as_ptr(),
                                          c.n_votes(), Some(on_status), user)
    };
    if rc != ffi::COA_OK {
        let pair = unsafe { Box::from_raw(user as *mut (oneshot::Sender<CertificateReply>, CertificateCrypto)) };
        let (sender, crypto) = *pair;
        let _ = sender.send(Err((rc, crypto)));
    }
}

fn submit_digest(queue: &Queue, bytes: Vec<u8>, sender: oneshot::Sender<DigestReply>) {
    // the bytes ride along with the sender and come back with the digest
    let user = Box::into_raw(Box::new((sender, bytes))) as *mut c_void;
    let (ptr, len) = unsafe {
        let pair = &*(user as *const (oneshot::Sender<DigestReply>, Vec<u8>));
        (pair.1.as_ptr(), pair.1.len())
    };
    let rc = unsafe { ffi::coa_queue_submit_digest(queue.0, ptr, len, Some(on_digest), user) };
    if rc != ffi::COA_OK {
        let pair = unsafe { Box::from_raw(user as *mut (oneshot::Sender<DigestReply>, Vec<u8>)) };
        let (sender, bytes) = *pair;
        let _ = sender.send(Err((rc, bytes)));
    }
}

// ------------------------------------------------------------- callbacks
// coa_verdict_cb: void (*)(void* user, int status, const uint8_t* verdicts,
// size_t n).  Each runs exactly once per queued request, on the engine's
// completion thread; `user` is the boxed sender(s) given at submission.

/// A coalesced window of `Signature::verify` requests: n verdict bytes, in
/// the order of the senders.
unsafe extern "C" fn on_verdicts(user: *mut c_void, status: c_int, verdicts: *const u8, n: usize) {
    let senders = Box::from_raw(user as *mut Vec<oneshot::Sender<Verdict>>);
    if status != ffi::COA_OK || verdicts.is_null() || n != senders.len() {
        let failure = if status != ffi::COA_OK { status } else { ffi::COA_EINVAL };
        for sender in *senders {
            let _ = sender.send(Err(failure));
        }
        return;
    }
    let bytes = std::slice::from_raw_parts(verdicts, n);
    for (sender, &byte) in senders.into_iter().zip(bytes) {
        let _ = sender.send(Ok(verdict_of(byte)));
    }
}

/// One vote batch: one verdict byte (the votes handed back on a failure).
unsafe extern "C" fn on_batch(user: *mut c_void, status: c_int, verdicts: *const u8, n: usize) {
    let pair = Box::from_raw(user as *mut (oneshot::Sender<BatchReply>, Vec<(PublicKey, [u8; 64])>));
    let (sender, votes) = *pair;
    let reply = if status != ffi::COA_OK {
        Err((status, votes))
    } else if verdicts.is_null() || n != 1 {
        Err((ffi::COA_EINVAL, votes))
    } else {
        Ok(verdict_of(*verdicts))
    };
    let _ = sender.send(reply);
}

/// One certificate: one status byte of COA_CERT_* bits, and the request
/// handed back.
unsafe extern "C" fn on_status(user: *mut c_void, status: c_int, verdicts: *const u8, n: usize) {
    let pair = Box::from_raw(user as *mut (oneshot::Sender<CertificateReply>, CertificateCrypto));
    let (sender, crypto) = *pair;
    let reply = if status != ffi::COA_OK {
        Err((status, crypto))
    } else if verdicts.is_null() || n != 1 {
        Err((ffi::COA_EINVAL, crypto))
    } else {
        Ok((*verdicts, crypto))
    };
    let _ = sender.send(reply);
}

/// One worker batch: the 32-byte Digest, and the batch handed back.
unsafe extern "C" fn on_digest(user: *mut c_void, status: c_int, verdicts: *const u8, n: usize) {
    let pair = Box::from_raw(user as *mut (oneshot::Sender<DigestReply>, Vec<u8>));
    let (sender, bytes) = *pair;
    let reply = if status != ffi::COA_OK {
        Err((status, bytes))
    } else if verdicts.is_null() || n != 32 {
        Err((ffi::COA_EINVAL, bytes))
    } else {
        let mut digest = [0u8; 32];
        digest.copy_from_slice(std::slice::from_raw_parts(verdicts, 32));
        Ok((Digest(digest), bytes))
    };
    let _ = sender.send(reply);
}

/// The process's service (created on first use, inside the tokio runtime):
/// for callers whose constructors take no service handle -- the worker's
/// `Processor::spawn` keeps the reference's signature this way.
/// COA_SERVICE_MAX_BATCH / COA_SERVICE_MAX_DELAY_US tune it.  Set up through
/// `std::sync::Once` (no `OnceLock`: the reference pins Rust 1.51.0).
pub fn global() -> VerifyService {
    static INIT: std::sync::Once = std::sync::Once::new();
    static mut SERVICE: *const VerifyService = std::ptr::null();
    unsafe {
        INIT.call_once(|| {
            let batch = std::env::var("COA_SERVICE_MAX_BATCH").ok().and_then(|v| v.parse().ok()).unwrap_or(65_536);
            let delay = std::env::var("COA_SERVICE_MAX_DELAY_US").ok().and_then(|v| v.parse().ok()).unwrap_or(500);
            SERVICE = Box::into_raw(Box::new(VerifyService::new(batch, delay)));
        });
        (*SERVICE).clone()
    }
}
