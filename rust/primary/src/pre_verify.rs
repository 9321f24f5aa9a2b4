//! The pre-verification stage between
//! `PrimaryReceiverHandler::dispatch` (primary/src/primary.rs:223-244) and
//! `Core` (primary/src/core.rs:349-389).
//!
//! `Core::run` takes one message at a time and its `sanitize_*` calls verify
//! each one synchronously (core.rs:306-346): one engine launch per header,
//! vote and certificate, where the engine's throughput comes from many
//! signatures per launch.  This task sits on the channel in front of `Core`:
//! every message the receiver delivers is submitted at once to the
//! `VerifyService` (the engine's aggregation queue, which coalesces the
//! requests of the window into a few launches), and each message is passed
//! on to `Core` as soon as its verdict is in AND every earlier message with
//! the same CLAIMED author has been passed on (the message's own author
//! field, read before it is verified; for a certificate the header's author).
//! That is neither the connection order nor the round-3 stage's global FIFO:
//! a certificate the `Helper` sends in reply to a `CertificatesRequest`
//! arrives over the replying peer's connection yet is ordered behind its
//! header author's messages, and a message that lies about its author can
//! only hold back (never reorder or change the verdict of) that author's
//! later messages, by at most its own verification time.  `Core` does not
//! depend on any order across authors or connections: the reference's
//! network interleaves peers arbitrarily on `Core`'s one channel, the
//! `Helper`'s replies come over other connections, and `Core` waits for
//! missing parents through its synchronizer whatever the arrival order
//! (primary/src/core.rs:276-303, synchronizer.rs).  A slow request -- a
//! certificate with a key outside the registered committee, or one the
//! exact random-linear-combination check re-decides (0.35-1.4 ms) --
//! therefore holds back only its claimed author's later messages, not every
//! message behind it (bench.py secondary.queue_round_mix.adversarial
//! measures both orderings; tests/test_pre_verify_host.py covers forwarded
//! certificates interleaved with the forwarding peer's headers).
//!
//! `Core` is not changed.  Its verify calls find the verdicts this stage
//! computed in `crypto::verified`, keyed by every byte the verdict depends on
//! (rust/crypto/src/verified.rs), so they return exactly what the engine
//! returns for those bytes -- Ok and Err alike, so `Core` never launches for
//! a message this stage saw, even under a flood of bad signatures -- and
//! `Core` raises the reference's `DagError`s in the reference's order,
//! because the non-crypto checks (gc round, expected vote, stake, worker
//! ids, quorum) still run there first.
//!
//! Wiring in primary/src/primary.rs (`Primary::spawn`):
//!     let (tx_pre_verify, rx_pre_verify) = channel(CHANNEL_CAPACITY);
//!     // the receiver handler sends to tx_pre_verify instead of
//!     // tx_primary_messages
//!     PreVerifier::spawn(crypto::service::global(), rx_pre_verify, tx_primary_messages);
//! and `mod pre_verify;` in primary/src/lib.rs.
use crate::gpu_certificate::certificate_crypto;
use crate::primary::PrimaryMessage;
use crypto::gpu::signature_bytes;
use crypto::service::VerifyService;
use crypto::{verified, Hash as _, PublicKey};
use futures::stream::{FuturesUnordered, StreamExt as _};
use std::collections::{HashMap, VecDeque};
use tokio::sync::mpsc::{Receiver, Sender};

/// Most messages between the receiver and `Core` at once (bounded memory;
/// beyond it the stage stops reading and the receiver's channel applies
/// back-pressure, as `Core`'s own channel does in the reference).
const MAX_IN_FLIGHT: usize = 16_384;

pub struct PreVerifier;

/// The message's claimed author (the order this stage keeps; unauthenticated
/// until the message is verified -- see the module doc).
fn author_of(message: &PrimaryMessage) -> PublicKey {
    match message {
        PrimaryMessage::Header(header) => header.author,
        PrimaryMessage::Vote(vote) => vote.author,
        PrimaryMessage::Certificate(certificate) => certificate.header.author,
        PrimaryMessage::CertificatesRequest(_, requestor) => *requestor,
    }
}

impl PreVerifier {
    pub fn spawn(service: VerifyService, mut rx_messages: Receiver<PrimaryMessage>, tx_core: Sender<PrimaryMessage>) {
        tokio::spawn(async move {
            let mut pending = FuturesUnordered::new();
            // per author: arrival sequence numbers in order, each with its
            // message once verified
            let mut lanes: HashMap<PublicKey, VecDeque<(u64, Option<PrimaryMessage>)>> = HashMap::new();
            let mut in_flight = 0usize;
            let mut seq = 0u64;
            loop {
                tokio::select! {
                    Some(message) = rx_messages.recv(), if in_flight < MAX_IN_FLIGHT => {
                        let author = author_of(&message);
                        seq += 1;
                        let my_seq = seq;
                        lanes.entry(author).or_default().push_back((my_seq, None));
                        in_flight += 1;
                        let service = service.clone();
                        pending.push(async move { (author, my_seq, pre_verify(service, message).await) });
                    },
                    Some((author, done_seq, message)) = pending.next() => {
                        let lane = lanes.get_mut(&author).expect("lane of a pending message");
                        if let Some(slot) = lane.iter_mut().find(|(s, _)| *s == done_seq) {
                            slot.1 = Some(message);
                        }
                        // release this author's verified prefix, in order
                        while lane.front().map_or(false, |(_, m)| m.is_some()) {
                            let (_, m) = lane.pop_front().unwrap();
                            in_flight -= 1;
                            tx_core
                                .send(m.unwrap())
                                .await
                                .expect("Failed to send message to the core");
                        }
                        if lane.is_empty() {
                            lanes.remove(&author);
                        }
                    },
                    else => break,
                }
            }
        });
    }
}

/// Verifies the crypto of one message through the service and remembers the
/// verdict -- Ok or Err -- for `Core`'s call; hands the message back
/// unchanged.
async fn pre_verify(service: VerifyService, message: PrimaryMessage) -> PrimaryMessage {
    match &message {
        PrimaryMessage::Header(header) => {
            // Header::verify's signature step (messages.rs:64-66)
            let signature = signature_bytes(&header.signature);
            let ok = service.verify(&header.id, &header.author, signature).await.is_ok();
            verified::remember_signature(&header.id, &header.author, &signature, ok);
        }
        PrimaryMessage::Vote(vote) => {
            // Vote::verify's signature step (messages.rs:139-141)
            let digest = vote.digest();
            let signature = signature_bytes(&vote.signature);
            let ok = service.verify(&digest, &vote.author, signature).await.is_ok();
            verified::remember_signature(&digest, &vote.author, &signature, ok);
        }
        PrimaryMessage::Certificate(certificate) => {
            // the crypto of Certificate::verify (messages.rs:189-215), fused;
            // the request comes back and becomes the cache key as it is
            let (bits, crypto) = service.certificate(certificate_crypto(certificate)).await;
            verified::remember_certificate(crypto.into_key(), bits);
        }
        PrimaryMessage::CertificatesRequest(..) => {}
    }
    message
}
