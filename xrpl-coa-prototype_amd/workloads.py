"""Synthetic, seeded inputs in the reference's byte formats.

* key seeds   seed_i = SHA512("coa-key" || u64le(i))[..32]
* messages    M_i = SHA512(u64le(i))[..32]  (the crypto API signs 32-byte Digests)
* worker batch  bincode WorkerMessage::Batch (worker/src/worker.rs:36-40) of
  977 x 512 B transactions formatted as node/src/benchmark_client.rs:117-130
  (tag byte, u64 big-endian counter, zero pad) = 508,052 bytes
* digest inputs of Header / Vote / Certificate (primary/src/messages.rs:70-84,
  145-153, 226-234)

Pure byte formatting (hashlib for the seeds); no verification logic here.
"""
import hashlib
import struct

import numpy as np

TX_SIZE = 512
TXS_PER_BATCH = 977  # first count with sum >= batch_size 500,000 (config/src/lib.rs:92)


def key_seeds(n, start=0):
    return np.frombuffer(b"".join(hashlib.sha512(b"coa-key" + struct.pack("<Q", i)).digest()[:32]
                                  for i in range(start, start + n)), np.uint8).reshape(n, 32).copy()


def messages(n, start=0):
    return np.frombuffer(b"".join(hashlib.sha512(struct.pack("<Q", i)).digest()[:32]
                                  for i in range(start, start + n)), np.uint8).reshape(n, 32).copy()


def worker_batch(b, ntx=TXS_PER_BATCH, size=TX_SIZE):
    """bincode(WorkerMessage::Batch(txs)): u32 variant 0 | u64 count | (u64 len | tx)*."""
    out = bytearray(struct.pack("<IQ", 0, ntx))
    for t in range(ntx):
        counter = b * ntx + t
        tag = 0 if t == 0 else 1  # one sample tx per burst, the rest standard
        tx = bytes([tag]) + struct.pack(">Q", counter)
        out += struct.pack("<Q", size) + tx + bytes(size - len(tx))
    return bytes(out)


def header_digest_input(author, round_, payload, parents):
    """Header::digest bytes: author | round u64 LE | (digest | worker_id u32 LE)* | parent*.
    payload: iterable of (digest32, worker_id) in BTreeMap (sorted) order."""
    out = bytearray(bytes(author)) + struct.pack("<Q", round_)
    for d, wid in sorted(payload, key=lambda x: bytes(x[0])):
        out += bytes(d) + struct.pack("<I", wid)
    for p in sorted(bytes(x) for x in parents):
        out += p
    return bytes(out)


def vote_digest_input(header_id, round_, origin):
    """Vote::digest == Certificate::digest bytes: id | round u64 LE | origin."""
    return bytes(header_id) + struct.pack("<Q", round_) + bytes(origin)
