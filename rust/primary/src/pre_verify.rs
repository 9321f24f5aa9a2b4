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
//! requests of the window into a few launches), and the messages are passed
//! on to `Core` in ARRIVAL ORDER as soon as each one's verdict is in (an
//! ordered set of futures: a later message never overtakes an earlier one).
//!
//! `Core` is not changed.  Its verify calls find the verdicts this stage
//! computed in `crypto::verified`, keyed by every byte the verdict depends on
//! (rust/crypto/src/verified.rs), so they return exactly what the engine
//! returns for those bytes -- and `Core` raises the reference's `DagError`s
//! in the reference's order, because the non-crypto checks (gc round,
//! expected vote, stake, worker ids, quorum) still run there first.  A
//! message whose signature fails here is simply not remembered: `Core`'s
//! call then asks the engine again and gets the same Err.
//!
//! Wiring in primary/src/primary.rs (`Primary::spawn`):
//!     let (tx_pre_verify, rx_pre_verify) = channel(CHANNEL_CAPACITY);
//!     // the receiver handler sends to tx_pre_verify instead of
//!     // tx_primary_messages
//!     PreVerifier::spawn(crypto::service::global(), rx_pre_verify, tx_primary_messages);
//! and `mod pre_verify;` in primary/src/lib.rs.
use crate::gpu_certificate::{certificate_crypto, signature_bytes};
use crate::primary::PrimaryMessage;
use crypto::service::VerifyService;
use crypto::{verified, Hash as _};
use futures::stream::{FuturesOrdered, StreamExt as _};
use tokio::sync::mpsc::{Receiver, Sender};

/// Most messages between the receiver and `Core` at once (bounded memory;
/// beyond it the stage stops reading and the receiver's channel applies
/// back-pressure, as `Core`'s own channel does in the reference).
const MAX_IN_FLIGHT: usize = 16_384;

pub struct PreVerifier;

impl PreVerifier {
    pub fn spawn(service: VerifyService, mut rx_messages: Receiver<PrimaryMessage>, tx_core: Sender<PrimaryMessage>) {
        tokio::spawn(async move {
            let mut pending = FuturesOrdered::new();
            loop {
                tokio::select! {
                    Some(message) = rx_messages.recv(), if pending.len() < MAX_IN_FLIGHT => {
                        pending.push_back(pre_verify(service.clone(), message));
                    },
                    Some(message) = pending.next() => {
                        tx_core
                            .send(message)
                            .await
                            .expect("Failed to send message to the core");
                    },
                    else => break,
                }
            }
        });
    }
}

/// Verifies the crypto of one message through the service and remembers the
/// verdict for `Core`'s call; hands the message back unchanged.
async fn pre_verify(service: VerifyService, message: PrimaryMessage) -> PrimaryMessage {
    match &message {
        PrimaryMessage::Header(header) => {
            // Header::verify's signature step (messages.rs:64-66)
            let signature = signature_bytes(&header.signature);
            if service.verify(&header.id, &header.author, signature).await.is_ok() {
                verified::remember_signature(&header.id, &header.author, &signature);
            }
        }
        PrimaryMessage::Vote(vote) => {
            // Vote::verify's signature step (messages.rs:139-141)
            let digest = vote.digest();
            let signature = signature_bytes(&vote.signature);
            if service.verify(&digest, &vote.author, signature).await.is_ok() {
                verified::remember_signature(&digest, &vote.author, &signature);
            }
        }
        PrimaryMessage::Certificate(certificate) => {
            // the crypto of Certificate::verify (messages.rs:189-215), fused
            let crypto = certificate_crypto(certificate);
            let key = crypto.key_bytes();
            let bits = service.certificate(crypto).await;
            verified::remember_certificate(key, bits);
        }
        PrimaryMessage::CertificatesRequest(..) => {}
    }
    message
}
