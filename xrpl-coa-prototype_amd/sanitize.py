"""Host mirror of the primary's pre-processing of incoming messages
 and of the worker's batch Processor (row a11), over
the engine's batched C ABI.

    Core::sanitize_header / _vote / _certificate   primary/src/core.rs:306-346
    Core::run dispatch                             primary/src/core.rs:349-389
    PrimaryReceiverHandler::dispatch (decode)      primary/src/primary.rs:223-244
    Processor::spawn                               worker/src/processor.rs:35-55

`Core.sanitize_*` keep the reference's checks and order (gc/round window,
expected-vote match, then the verify wrappers of certificates.py) and raise
the same DagError kinds.

`Core.sanitize_frames` is the pre-verification stage SURVEY 8(f) f1 asks
for: a window of bincode `PrimaryMessage` frames is decoded natively
(coa_wire_*), every certificate's crypto runs in ONE fused launch
(coa_certificate_verify_many), headers and votes in one verify_strict launch
each (their digests in one SHA-512 launch), and each frame gets the result
Core::run would have produced for it alone, in order.  The reference's Core
handles one message at a time; nothing here changes a verdict, only how many
signatures share a launch.

`Processor` hashes serialized WorkerMessage::Batch buffers on the device
(one launch per window), stores them and emits the bincode of
WorkerPrimaryMessage::{OurBatch, OthersBatch}(digest, worker id).
"""
import struct

import numpy as np

import certificates as C
import coa_crypto
from coa_crypto import Digest, PublicKey, Signature


class TooOld(C.DagError):
    pass


class UnexpectedVote(C.DagError):
    pass


class SerializationError(C.DagError):
    pass


class Core:
    """The verification-relevant state of primary::Core: the committee, the
    garbage-collection round and the header we are collecting votes for."""

    def __init__(self, committee, gc_round=0, current_header=None):
        self.committee = committee
        self.gc_round = gc_round
        self.current_header = current_header or C.Header()

    # primary/src/core.rs:306-317
    def sanitize_header(self, header):
        if not self.gc_round <= header.round:
            raise TooOld(header.id, header.round)
        header.verify(self.committee)

    # primary/src/core.rs:319-336
    def sanitize_vote(self, vote):
        h = self.current_header
        if not h.round <= vote.round:
            raise TooOld(vote.digest(), vote.round)
        if not (vote.id == h.id and vote.origin == h.author and vote.round == h.round):
            raise UnexpectedVote(vote.id)
        vote.verify(self.committee)

    # primary/src/core.rs:338-346
    def sanitize_certificate(self, certificate):
        if not self.gc_round <= certificate.round():
            raise TooOld(certificate.digest(), certificate.round())
        certificate.verify(self.committee)

    # ------------------------------------------------------------------
    def sanitize_frames(self, frames, rng_seed=0):
        """Pre-verify a window of PrimaryMessage frames.  Returns, per frame,
        (kind, None | DagError): kind is coa_crypto.MSG_* (or None when the
        frame does not decode, with a SerializationError)."""
        n = len(frames)
        kinds, _, _ = coa_crypto.wire_scan(frames)
        out = [None] * n
        idx = {k: [i for i in range(n) if kinds[i] == k]
               for k in (coa_crypto.MSG_HEADER, coa_crypto.MSG_VOTE, coa_crypto.MSG_CERTIFICATE)}
        for i in range(n):
            if kinds[i] < 0:
                out[i] = (None, SerializationError(int(kinds[i])))
            elif kinds[i] == coa_crypto.MSG_CERT_REQUEST:
                out[i] = (coa_crypto.MSG_CERT_REQUEST, None)  # routed to the helper, no crypto
        self._certificates([frames[i] for i in idx[coa_crypto.MSG_CERTIFICATE]], idx[coa_crypto.MSG_CERTIFICATE],
                           out, rng_seed)
        self._headers([frames[i] for i in idx[coa_crypto.MSG_HEADER]], idx[coa_crypto.MSG_HEADER], out)
        self._votes([frames[i] for i in idx[coa_crypto.MSG_VOTE]], idx[coa_crypto.MSG_VOTE], out)
        return out

    def _certificates(self, frames, where, out, rng_seed):
        if not frames:
            return
        d = coa_crypto.wire_decode_certificates(frames)
        st = coa_crypto.certificate_verify_many(d["header_inputs"], d["ids"], d["origins"], d["header_sigs"],
                                                d["rounds"], d["vote_pks"], d["vote_sigs"], d["vote_offsets"],
                                                rng_seed=rng_seed)
        for j, i in enumerate(where):
            cert = _certificate_from(d, j)
            err = None
            try:
                if not self.gc_round <= cert.round():
                    raise TooOld(cert.digest(), cert.round())
                if not cert.is_genesis(self.committee):
                    C._raise_in_order(cert, self.committee, int(st[j]))
            except C.DagError as e:
                err = e
            out[i] = (coa_crypto.MSG_CERTIFICATE, err)

    def _headers(self, frames, where, out):
        if not frames:
            return
        d = coa_crypto.wire_decode_headers(frames)
        digests = coa_crypto.sha512_many(d["header_inputs"])[:, :32]
        bad_sig = coa_crypto.verify_strict_many(d["ids"], d["authors"], d["sigs"])
        for j, i in enumerate(where):
            h = _header_from(d, j)
            err = None
            try:
                if not self.gc_round <= h.round:
                    raise TooOld(h.id, h.round)
                # Header::verify (primary/src/messages.rs:48-67), its order
                if bytes(digests[j]) != bytes(h.id):
                    raise C.InvalidHeaderId(h.id)
                if self.committee.stake(h.author) <= 0:
                    raise C.UnknownAuthority(h.author)
                for wid in h.payload.values():
                    if not self.committee.has_worker(h.author, wid):
                        raise C.MalformedHeader(h.id)
                if bad_sig[j]:
                    raise C.InvalidSignature()
            except C.DagError as e:
                err = e
            out[i] = (coa_crypto.MSG_HEADER, err)

    def _votes(self, frames, where, out):
        if not frames:
            return
        d = coa_crypto.wire_decode_votes(frames)
        vin = [bytes(d["ids"][j]) + struct.pack("<Q", int(d["rounds"][j])) + bytes(d["origins"][j])
               for j in range(len(frames))]
        digests = coa_crypto.sha512_many(vin)[:, :32].copy()
        bad_sig = coa_crypto.verify_strict_many(digests, d["authors"], d["sigs"])
        h = self.current_header
        for j, i in enumerate(where):
            err = None
            vid, vround = Digest(bytes(d["ids"][j])), int(d["rounds"][j])
            origin, author = PublicKey(bytes(d["origins"][j])), PublicKey(bytes(d["authors"][j]))
            try:
                if not h.round <= vround:
                    raise TooOld(Digest(bytes(digests[j])), vround)
                if not (vid == h.id and origin == h.author and vround == h.round):
                    raise UnexpectedVote(vid)
                if self.committee.stake(author) <= 0:                     # Vote::verify, messages.rs:131-142
                    raise C.UnknownAuthority(author)
                if bad_sig[j]:
                    raise C.InvalidSignature()
            except C.DagError as e:
                err = e
            out[i] = (coa_crypto.MSG_VOTE, err)


def _payload_from_input(hi, n_payload):
    pay = {}
    for k in range(n_payload):
        o = 40 + 36 * k
        pay[Digest(hi[o:o + 32])] = struct.unpack_from("<I", hi, o + 32)[0]
    parents = {Digest(hi[o:o + 32]) for o in range(40 + 36 * n_payload, len(hi), 32)}
    return pay, parents


def _header_from(d, j):
    hi = d["header_inputs"][j]
    pay, parents = _payload_from_input(hi, int(d["payload_counts"][j]))
    author = d["authors"][j] if "authors" in d else d["origins"][j]
    sig = d["sigs"][j] if "sigs" in d else d["header_sigs"][j]
    h = C.Header(PublicKey(bytes(author)), int(d["rounds"][j]), pay, parents, Digest(bytes(d["ids"][j])),
                 Signature.from_bytes(bytes(sig)))
    h._digest_input = hi
    return h


def _certificate_from(d, j):
    lo, hi = int(d["vote_offsets"][j]), int(d["vote_offsets"][j + 1])
    votes = [(PublicKey(bytes(d["vote_pks"][k])), Signature.from_bytes(bytes(d["vote_sigs"][k])))
             for k in range(lo, hi)]
    return C.Certificate(_header_from(d, j), votes)


# ---------------------------------------------------------------------------
def message_author(message):
    """The message's claimed author (a certificate's: its header author):
    the order the pre-verification stage keeps (rust/primary/src/pre_verify.rs
    author_of).  Not the delivering connection -- a certificate forwarded by
    another peer's Helper is ordered behind its header author's messages --
    and unauthenticated until verified; Core depends on no cross-author
    order (see pre_verify.rs's module doc)."""
    if isinstance(message, C.Certificate):
        return message.origin()
    return message.author


class PreVerifier:
    """Mirror of rust/primary/src/pre_verify.rs: the stage between
    PrimaryReceiverHandler::dispatch (primary/src/primary.rs:223-244) and
    Core (primary/src/core.rs:349-389).  A window of Header / Vote /
    Certificate messages has its crypto verified in coalesced engine calls --
    every header and vote signature in ONE verify_strict_many call, every
    certificate in ONE certificate_verify_many call -- and every verdict, Ok
    and Err alike, is remembered in coa_crypto.verified, where Core's
    unchanged one-at-a-time calls (Header.verify, Vote.verify,
    Certificate.verify) find it: Core then makes no engine call for any
    message the stage saw.  `verify_many` / `certificate_many` default to the
    engine's entry points (tests pass counting stand-ins)."""

    def __init__(self, verify_many=None, certificate_many=None):
        self.verify_many = verify_many or coa_crypto.verify_strict_many
        self.certificate_many = certificate_many or coa_crypto.certificate_verify_many

    def window(self, messages):
        messages = list(messages)
        trip, certs = [], []
        for m in messages:
            if isinstance(m, C.Header):                    # Header::verify's signature (messages.rs:64-66)
                trip.append((bytes(m.id), bytes(m.author), m.signature.flatten()))
            elif isinstance(m, C.Vote):                    # Vote::verify's signature (messages.rs:139-141)
                trip.append((bytes(m.digest()), bytes(m.author), m.signature.flatten()))
            elif isinstance(m, C.Certificate) and m.header is not None:
                certs.append(m)
        if trip:
            arr = [np.frombuffer(b"".join(t[i] for t in trip), np.uint8).reshape(len(trip), -1) for i in range(3)]
            bad = self.verify_many(*arr)
            for (d, k, sg), b in zip(trip, bad):
                coa_crypto.verified.remember_signature(d, k, sg, int(b) == 0)
        if certs:
            hdr = [c.header for c in certs]
            offs = np.zeros(len(certs) + 1, np.uint64)
            offs[1:] = np.cumsum([len(c.votes) for c in certs])
            vp = np.frombuffer(b"".join(bytes(pk) for c in certs for pk, _ in c.votes), np.uint8).reshape(-1, 32)
            vs = np.frombuffer(b"".join(sg.flatten() for c in certs for _, sg in c.votes), np.uint8).reshape(-1, 64)
            st = self.certificate_many([h.digest_input() for h in hdr],
                                       np.frombuffer(b"".join(bytes(h.id) for h in hdr), np.uint8).reshape(-1, 32),
                                       np.frombuffer(b"".join(bytes(h.author) for h in hdr), np.uint8).reshape(-1, 32),
                                       np.frombuffer(b"".join(h.signature.flatten() for h in hdr),
                                                     np.uint8).reshape(-1, 64),
                                       np.array([h.round for h in hdr], np.uint64), vp, vs, offs)
            for c, b in zip(certs, st):
                coa_crypto.verified.remember_certificate(c.crypto_key(), int(b))
        return messages


def release_times(arrival_s, done_s, authors, per_author=True):
    """When the pre-verification stage hands each message to Core, given when
    it arrived, when its verdict came back and who sent it: as soon as its
    verdict is in and every earlier message -- of the same author
    (rust/primary/src/pre_verify.rs, per_author=True) or of anyone (the
    round-3 stage's one FuturesOrdered, per_author=False) -- has been handed
    on.  Messages are in arrival order."""
    out = [0.0] * len(done_s)
    last = {}
    prev = float("-inf")
    for i, (t, a) in enumerate(zip(done_s, authors)):
        gate = last.get(a, float("-inf")) if per_author else prev
        out[i] = max(t, gate, arrival_s[i])
        last[a] = out[i]
        prev = out[i]
    return out


class Processor:
    """worker::Processor (worker/src/processor.rs:21-55): hash, store, emit
    the digest message.  `process` takes a window of serialized
    WorkerMessage::Batch buffers and hashes them in one device launch."""

    OUR_BATCH, OTHERS_BATCH = 0, 1  # WorkerPrimaryMessage variants (primary/src/primary.rs:51-56)

    def __init__(self, worker_id, store, own_digest=True):
        self.id = worker_id
        self.store = store
        self.own_digest = own_digest

    def process(self, batches):
        if not batches:
            return []
        digests = coa_crypto.sha512_many(list(batches))[:, :32]
        variant = self.OUR_BATCH if self.own_digest else self.OTHERS_BATCH
        out = []
        for b, d in zip(batches, digests):
            self.store[bytes(d)] = bytes(b)                               # store.write(digest, batch)
            out.append(struct.pack("<I", variant) + bytes(d) + struct.pack("<I", self.id))  # bincode
        return out
