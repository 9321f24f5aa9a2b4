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


# ---------------------------------------------------------------------------
# C5 adversarial mix: byte-level mutations of valid triples.
# Expected verdicts are never computed here -- they come from the oracle in
# the tests.
L_ORDER = 2 ** 252 + 27742317777372353535851937790883648493
P_FIELD = 2 ** 255 - 19

SMALL_ORDER = [bytes.fromhex(h) for h in (
    "0100000000000000000000000000000000000000000000000000000000000000",
    "0100000000000000000000000000000000000000000000000000000000000080",
    "eeffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f",
    "eeffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff",
    "c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a",
    "c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac03fa",
    "0000000000000000000000000000000000000000000000000000000000000000",
    "0000000000000000000000000000000000000000000000000000000000000080",
    "edffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f",
    "edffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff",
    "26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05",
    "26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc85",
    "ecffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f",
    "ecffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff",
)]
# y in [p, p+18] that decode to points of large order (accepted by dalek's
# decompression, so only the equation can reject them)
NONCANONICAL = [((y + P_FIELD) | (s << 255)).to_bytes(32, "little")
                for y in (3, 4, 5, 6, 9, 10, 14, 15, 16, 18) for s in (0, 1)]
OFF_CURVE = [y.to_bytes(32, "little") for y in (2, 7, 8, 11, 12, 13, 17, 20)]

ADVERSARIAL_CLASSES = ("s_plus_l", "s_high_bit", "noncanonical_R", "small_order_R", "small_order_A",
                       "off_curve", "bitflip", "mixed_order_A")


def adversarial_mix(msgs, pks, sigs, frac=0.01, seed=0xC0A5, mixed_pool=None):
    """Mutate `frac` of the items (indices from a seeded shuffle), split evenly
    over the 8 classes of SURVEY 8(d).  mixed_pool: list of (msg, pk, sig)
    mixed-order triples (class 8, accepted by cofactorless dalek).
    Returns (msgs, pks, sigs, class_of) with class_of[i] = -1 for untouched."""
    msgs, pks, sigs = msgs.copy(), pks.copy(), sigs.copy()
    n = pks.shape[0]
    rng = np.random.default_rng(seed)
    k = int(round(n * frac))
    idx = rng.permutation(n)[:k]
    cls = np.full(n, -1, np.int8)
    for j, i in enumerate(idx):
        c = j % (8 if mixed_pool else 7)
        cls[i] = c
        r = int(rng.integers(0, 1 << 30))
        if c == 0:  # s + l
            s = int.from_bytes(bytes(sigs[i, 32:]), "little") + L_ORDER
            sigs[i, 32:] = np.frombuffer(s.to_bytes(32, "little"), np.uint8)
        elif c == 1:  # bit 255/254/253/252 of s
            sigs[i, 63] |= (0x80, 0x40, 0x20, 0x10)[r % 4]
        elif c == 2:  # y >= p encodings of R
            sigs[i, :32] = np.frombuffer(NONCANONICAL[r % len(NONCANONICAL)], np.uint8)
        elif c == 3:
            sigs[i, :32] = np.frombuffer(SMALL_ORDER[r % len(SMALL_ORDER)], np.uint8)
        elif c == 4:
            pks[i] = np.frombuffer(SMALL_ORDER[r % len(SMALL_ORDER)], np.uint8)
        elif c == 5:
            enc = np.frombuffer(OFF_CURVE[r % len(OFF_CURVE)], np.uint8)
            if r & 1:
                sigs[i, :32] = enc
            else:
                pks[i] = enc
        elif c == 6:
            which = r % 3
            if which == 0:
                msgs[i, (r >> 2) % msgs.shape[1]] ^= 1 << ((r >> 8) % 8)
            elif which == 1:
                sigs[i, (r >> 2) % 32] ^= 1 << ((r >> 8) % 8)
            else:
                sigs[i, 32 + (r >> 2) % 31] ^= 1 << ((r >> 8) % 8)
        else:
            m, p, s = mixed_pool[r % len(mixed_pool)]
            msgs[i], pks[i], sigs[i] = (np.frombuffer(m, np.uint8), np.frombuffer(p, np.uint8),
                                        np.frombuffer(s, np.uint8))
    return msgs, pks, sigs, cls
