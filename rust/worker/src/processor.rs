// worker/src/processor.rs with the batch digests on the MI355X engine.
//
// The reference's `Processor` (worker/src/processor.rs:35-55) hashes one
// batch per loop iteration: receive, `Sha512::digest`, store, send.  On the
// GPU one 508 KB batch is a serial chain of 3,970 SHA-512 compressions
// (~14 ms per launch, however few batches it holds), so a per-batch launch
// would cap a worker at ~70 batches/s.  This version keeps the reference's
// signature and behaviour -- every batch is hashed, stored under its digest
// and announced to the primary, in arrival order -- but streams the batches:
// each received batch goes to the `VerifyService` at once (the engine's
// queue coalesces all pending batches, of both Processors, into one launch
// that hashes them in parallel), and an ordered set of futures releases the
// batches to the store and the primary in the order they arrived, while
// later batches are already on the GPU.  At C4's rate (1M tx/s of 512 B =
// ~1,000 batches/s per worker) the queue's windows carry the batches of the
// previous launch's ~14 ms, so one launch covers many batches and the rate
// is sustained with ~15-30 ms of added latency per batch (bench.py
// secondary.c4_stream measures it).
use crate::worker::SerializedBatchDigestMessage;
use config::WorkerId;
use futures::stream::{FuturesOrdered, StreamExt as _};
use primary::WorkerPrimaryMessage;
use store::Store;
use tokio::sync::mpsc::{Receiver, Sender};

#[cfg(test)]
#[path = "tests/processor_tests.rs"]
pub mod processor_tests;

/// Indicates a serialized `WorkerMessage::Batch` message.
pub type SerializedBatchMessage = Vec<u8>;

/// Batches hashed or being hashed and not yet stored (~128 MB at 508 KB).
const MAX_IN_FLIGHT: usize = 256;

/// Hashes and stores batches, it then outputs the batch's digest.
pub struct Processor;

impl Processor {
    pub fn spawn(
        // Our worker's id.
        id: WorkerId,
        // The persistent storage.
        mut store: Store,
        // Input channel to receive batches.
        mut rx_batch: Receiver<SerializedBatchMessage>,
        // Output channel to send out batches' digests.
        tx_digest: Sender<SerializedBatchDigestMessage>,
        // Whether we are processing our own batches or the batches of other nodes.
        own_digest: bool,
    ) {
        tokio::spawn(async move {
            let service = crypto::service::global();
            let mut hashing = FuturesOrdered::new();
            loop {
                tokio::select! {
                    // Hash the batch: handed to the engine's queue at once.
                    Some(batch) = rx_batch.recv(), if hashing.len() < MAX_IN_FLIGHT => {
                        hashing.push_back(service.digest(batch));
                    },
                    // The oldest batch is hashed: store it and deliver its digest.
                    Some((digest, batch)) = hashing.next() => {
                        store.write(digest.to_vec(), batch).await;
                        let message = match own_digest {
                            true => WorkerPrimaryMessage::OurBatch(digest, id),
                            false => WorkerPrimaryMessage::OthersBatch(digest, id),
                        };
                        let message = bincode::serialize(&message)
                            .expect("Failed to serialize our own worker-primary message");
                        tx_digest
                            .send(message)
                            .await
                            .expect("Failed to send digest");
                    },
                    else => break,
                }
            }
        });
    }
}
