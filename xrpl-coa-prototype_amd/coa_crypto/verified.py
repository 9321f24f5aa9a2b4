"""Verdicts computed ahead of the synchronous call that asks for them -- the
Python mirror of rust/crypto/src/verified.rs.

The pre-verification stage (sanitize.PreVerifier; rust/primary/src/
pre_verify.rs) verifies the messages the receiver hands to Core in coalesced
launches before Core sees them.  Core is unchanged: Header.verify /
Vote.verify reach Signature.verify and Certificate.verify reaches the fused
certificate call, and both look here first.

Exactness: a signature entry is keyed by all 128 bytes (digest, key, R || s)
its verify_strict verdict depends on, a certificate entry by every byte of
its crypto input (certificate_key), and BOTH outcomes are kept -- the verdict
is a pure function of those bytes, so a remembered Err is exactly as faithful
as a remembered Ok, and Core never asks the engine again for a message the
stage saw.  Entries are consumed by the lookup that uses them; the oldest are
dropped beyond a fixed capacity (FIFO), as in the Rust cache.
"""
import collections
import struct
import threading

SIGNATURES = 1 << 17
CERTIFICATES = 1 << 14


class _Fifo:
    def __init__(self, cap):
        self.cap = cap
        self.map = {}
        self.order = collections.deque()
        self.gen = 0
        self.lock = threading.Lock()

    def insert(self, key, value):
        with self.lock:
            g = self.gen
            self.gen += 1
            self.map[key] = (value, g)
            self.order.append((key, g))
            while len(self.order) > self.cap:
                old, og = self.order.popleft()
                if self.map.get(old, (None, None))[1] == og:
                    del self.map[old]

    def take(self, key):
        with self.lock:
            v = self.map.pop(key, None)
            return None if v is None else v[0]

    def clear(self):
        with self.lock:
            self.map.clear()
            self.order.clear()


_signatures = _Fifo(SIGNATURES)
_certificates = _Fifo(CERTIFICATES)


def _triple(digest, public_key, signature):
    k = bytes(digest) + bytes(public_key) + bytes(signature)
    if len(k) != 128:
        raise ValueError("digest, key and signature are 32 + 32 + 64 bytes")
    return k


def remember_signature(digest, public_key, signature, ok):
    """The engine's Signature::verify verdict of this triple (ok: Ok, else Err)."""
    _signatures.insert(_triple(digest, public_key, signature), bool(ok))


def take_signature(digest, public_key, signature):
    """True (Ok) / False (Err) remembered for exactly this triple, or None;
    the entry is consumed."""
    return _signatures.take(_triple(digest, public_key, signature))


def certificate_key(header_input, id_, origin, header_sig, round_, vote_pks, vote_sigs):
    """Every byte a certificate's crypto verdict depends on, length-framed --
    the layout of rust/crypto/src/service.rs CertificateCrypto:
    header_len u64 | header input | id | origin | header R || s | round u64 |
    n_votes u64 | keys | signatures."""
    hi = bytes(header_input)
    vp, vs = bytes(vote_pks), bytes(vote_sigs)
    n = len(vp) // 32
    if len(vp) != 32 * n or len(vs) != 64 * n:
        raise ValueError("32-byte keys and 64-byte signatures, one per vote")
    return (struct.pack("<Q", len(hi)) + hi + bytes(id_) + bytes(origin) + bytes(header_sig) +
            struct.pack("<QQ", int(round_), n) + vp + vs)


def remember_certificate(key, bits):
    _certificates.insert(bytes(key), int(bits))


def take_certificate(key):
    """The COA_CERT_* bits remembered for exactly this crypto input, or None
    (consumed)."""
    return _certificates.take(bytes(key))


def clear():
    """Drop every entry (tests)."""
    _signatures.clear()
    _certificates.clear()
