"""Host mirror of the reference's verify callers (primary/src/messages.rs) on
top of the engine's batched C ABI -- SURVEY.md 8(a) rows a7-a9.

    Header::digest / verify        primary/src/messages.rs:48-84
    Vote::digest / verify          primary/src/messages.rs:131-153
    Certificate::digest / verify   primary/src/messages.rs:175-234
    Committee::quorum_threshold    config/src/lib.rs:168-173 (2N/3 + 1 of stake)

`Certificate.verify` follows the reference's check order exactly and raises
the same error kinds (DagError variants, primary/src/error.rs).  Its crypto
(header digest, header signature, vote batch) is ONE engine call,
coa_certificate_verify (fused kernel over the registered committee's key
combs -- `Committee.register()`); the status bits it
returns are then consumed in the reference's order, interleaved with the
host-side protocol checks, so the error raised is the reference's.
`verify_stepwise` is the same method over the per-primitive entry points
(verify_strict / verify_batch / Digest), kept for cross-checks.
`verify_certificates` / `verify_certificate_batch` do the same for many
certificates with one coa_certificate_verify_many call.
"""
import struct

import numpy as np

import coa_crypto
from coa_crypto import Digest, PublicKey, Signature


class DagError(Exception):
    """primary::error::DagError kinds used by the verify paths."""


class InvalidHeaderId(DagError):
    pass


class UnknownAuthority(DagError):
    pass


class MalformedHeader(DagError):
    pass


class AuthorityReuse(DagError):
    pass


class CertificateRequiresQuorum(DagError):
    pass


class InvalidSignature(DagError):
    pass


class Committee:
    """config::Committee reduced to what the verify paths read: stake per
    authority and each authority's worker ids."""

    def __init__(self, stakes, workers=None):
        self.stakes = {PublicKey(bytes(k)): int(s) for k, s in stakes.items()}
        self.workers = {PublicKey(bytes(k)): set(w) for k, w in (workers or {}).items()}

    def stake(self, name):
        return self.stakes.get(name, 0)

    def quorum_threshold(self):
        total = sum(self.stakes.values())
        return 2 * total // 3 + 1

    def has_worker(self, name, worker_id):
        return worker_id in self.workers.get(name, {0})

    def authorities(self):
        return sorted(self.stakes)

    def register(self):
        """Hand the committee's keys to the engine's key cache (f2).  Needed
        for speed only: verdicts do not depend on it."""
        return coa_crypto.committee_register(np.array([list(bytes(k)) for k in self.authorities()], np.uint8))


class Header:
    def __init__(self, author=PublicKey(), round_=0, payload=None, parents=None, id_=Digest(), signature=None):
        self.author = author
        self.round = round_
        self.payload = dict(payload or {})  # Digest -> worker id (BTreeMap)
        self.parents = set(parents or ())   # BTreeSet<Digest>
        self.id = id_
        self.signature = signature or Signature()

    def digest_input(self):
        if getattr(self, "_digest_input", None) is not None:
            return self._digest_input
        out = bytearray(bytes(self.author)) + struct.pack("<Q", self.round)
        for d in sorted(self.payload, key=bytes):
            out += bytes(d) + struct.pack("<I", self.payload[d])
        for p in sorted(self.parents, key=bytes):
            out += bytes(p)
        return bytes(out)

    def digest(self):
        return coa_crypto.digest_many([self.digest_input()])[0]

    def verify(self, committee):
        if self.digest() != self.id:
            raise InvalidHeaderId(self.id)
        if committee.stake(self.author) <= 0:
            raise UnknownAuthority(self.author)
        for wid in self.payload.values():
            if not committee.has_worker(self.author, wid):
                raise MalformedHeader(self.id)
        try:
            self.signature.verify(self.id, self.author)
        except coa_crypto.CryptoError as e:
            raise InvalidSignature() from e


class Vote:
    def __init__(self, id_, round_, origin, author, signature=None):
        self.id, self.round, self.origin, self.author = id_, round_, origin, author
        self.signature = signature or Signature()

    def digest_input(self):
        return bytes(self.id) + struct.pack("<Q", self.round) + bytes(self.origin)

    def digest(self):
        return coa_crypto.digest_many([self.digest_input()])[0]

    def verify(self, committee):
        if committee.stake(self.author) <= 0:
            raise UnknownAuthority(self.author)
        try:
            self.signature.verify(self.digest(), self.author)
        except coa_crypto.CryptoError as e:
            raise InvalidSignature() from e


class Certificate:
    def __init__(self, header, votes):
        self.header = header
        self.votes = list(votes)  # [(PublicKey, Signature)]

    def round(self):
        return self.header.round

    def origin(self):
        return self.header.author

    def digest_input(self):
        return bytes(self.header.id) + struct.pack("<Q", self.round()) + bytes(self.origin())

    def digest(self):
        return coa_crypto.digest_many([self.digest_input()])[0]

    def is_genesis(self, committee):
        # Certificate::genesis(committee).contains(self): PartialEq compares
        # header id, round and origin (primary/src/messages.rs:249-256)
        return (self.header.id == Digest() and self.round() == 0
                and self.origin() in committee.stakes)

    def quorum_check(self, committee):
        weight, used = 0, set()
        for name, _ in self.votes:
            if name in used:
                raise AuthorityReuse(name)
            s = committee.stake(name)
            if s <= 0:
                raise UnknownAuthority(name)
            used.add(name)
            weight += s
        if weight < committee.quorum_threshold():
            raise CertificateRequiresQuorum()

    def verify(self, committee, rng_seed=0):
        """Certificate::verify (primary/src/messages.rs:189-215): one fused
        engine call for the crypto, checks raised in the reference's order."""
        if self.is_genesis(committee):
            return
        h = self.header
        # the bits the pre-verification stage computed for exactly these bytes
        # (coa_crypto.verified; rust/primary/src/gpu_certificate.rs), else one
        # engine call
        st = coa_crypto.verified.take_certificate(self.crypto_key())
        if st is None:
            vp = np.array([list(bytes(pk)) for pk, _ in self.votes], np.uint8).reshape(-1, 32)
            vs = np.array([list(sg.flatten()) for _, sg in self.votes], np.uint8).reshape(-1, 64)
            st = coa_crypto.certificate_verify(h.digest_input(), h.id, h.author, h.signature.flatten(), h.round, vp,
                                               vs, rng_seed=rng_seed)
        _raise_in_order(self, committee, st)

    def crypto_key(self):
        """Every byte the certificate's crypto verdict depends on
        (coa_crypto.verified.certificate_key)."""
        h = self.header
        return coa_crypto.verified.certificate_key(
            h.digest_input(), h.id, h.author, h.signature.flatten(), h.round,
            b"".join(bytes(pk) for pk, _ in self.votes), b"".join(sg.flatten() for _, sg in self.votes))

    def verify_stepwise(self, committee, rng_seed=0):
        """The same checks through the per-primitive entry points."""
        if self.is_genesis(committee):
            return
        self.header.verify(committee)
        self.quorum_check(committee)
        try:
            Signature.verify_batch(self.digest(), self.votes, rng_seed=rng_seed)
        except coa_crypto.CryptoError as e:
            raise InvalidSignature() from e


def _raise_in_order(cert, committee, st):
    """Apply Certificate::verify's checks in the reference's order, the crypto
    ones read from the engine's status bits (include/coa_verify.h)."""
    h = cert.header
    if st & coa_crypto.CERT_BAD_HEADER_ID:                      # messages.rs:49-51
        raise InvalidHeaderId(h.id)
    if committee.stake(h.author) <= 0:                          # :53-56
        raise UnknownAuthority(h.author)
    for wid in h.payload.values():                              # :58-62
        if not committee.has_worker(h.author, wid):
            raise MalformedHeader(h.id)
    if st & coa_crypto.CERT_BAD_HEADER_SIG:                     # :64-66
        raise InvalidSignature()
    cert.quorum_check(committee)                                # :196-211
    if st & coa_crypto.CERT_BAD_VOTES:                          # :214
        raise InvalidSignature()


def verify_certificates(certs, committee, rng_seed=0):
    """Certificate::verify for many certificates: the crypto of all of them in
    one coa_certificate_verify_many call, then the checks in the reference's
    order.  Returns a list with None (Ok) or the DagError instance."""
    n = len(certs)
    res = [None] * n
    todo = [i for i, c in enumerate(certs) if not c.is_genesis(committee)]
    if not todo:
        return res
    hs = [certs[i].header for i in todo]
    ids = np.array([list(bytes(h.id)) for h in hs], np.uint8)
    origins = np.array([list(bytes(h.author)) for h in hs], np.uint8)
    hsigs = np.array([list(h.signature.flatten()) for h in hs], np.uint8)
    rounds = np.array([h.round for h in hs], np.uint64)
    vp = np.array([list(bytes(pk)) for i in todo for pk, _ in certs[i].votes], np.uint8).reshape(-1, 32)
    vs = np.array([list(sg.flatten()) for i in todo for _, sg in certs[i].votes], np.uint8).reshape(-1, 64)
    offs = np.zeros(len(todo) + 1, np.uint64)
    offs[1:] = np.cumsum([len(certs[i].votes) for i in todo])
    st = coa_crypto.certificate_verify_many([h.digest_input() for h in hs], ids, origins, hsigs, rounds, vp, vs, offs,
                                            rng_seed=rng_seed)
    for j, i in enumerate(todo):
        try:
            _raise_in_order(certs[i], committee, int(st[j]))
        except DagError as e:
            res[i] = e
    return res


# ---------------------------------------------------------------------------
# Struct-of-arrays certificates for bulk runs (benchmark C1/C3 shapes).
class CertificateBatch:
    """n certificates as arrays: header digest inputs, ids, authors, header
    signatures, certificate digests and concatenated votes (group offsets)."""

    def __init__(self, header_inputs, ids, authors, header_sigs, cert_digests, vote_pks, vote_sigs, offsets,
                 voter_idx, author_idx, round_):
        self.round = round_
        self.header_inputs = header_inputs      # list of bytes (3,336 B at C3)
        self.ids = ids                          # uint8 [n, 32]
        self.authors = authors                  # uint8 [n, 32]
        self.header_sigs = header_sigs          # uint8 [n, 64]
        self.cert_digests = cert_digests        # uint8 [n, 32]
        self.vote_pks = vote_pks                # uint8 [nv, 32]
        self.vote_sigs = vote_sigs              # uint8 [nv, 64]
        self.offsets = offsets                  # uint64 [n + 1]
        self.voter_idx = voter_idx              # int [nv] key-seed index of each voter (synthesis only;
                                                # the checks read vote_pks)
        self.author_idx = author_idx            # int [n]

    def __len__(self):
        return self.ids.shape[0]

    def certificate(self, i):
        """Materialise certificate i as objects (tests / single verifies)."""
        lo, hi = int(self.offsets[i]), int(self.offsets[i + 1])
        votes = [(PublicKey(bytes(self.vote_pks[j])), Signature.from_bytes(bytes(self.vote_sigs[j])))
                 for j in range(lo, hi)]
        h = Header(PublicKey(bytes(self.authors[i])), self.round, {}, set(), Digest(bytes(self.ids[i])),
                   Signature.from_bytes(bytes(self.header_sigs[i])))
        h._digest_input = self.header_inputs[i]
        return Certificate(h, votes)


def synth_certificates(n_certs, committee_size=100, n_votes=None, n_payload=32, round_=1, seed=0, rotate=True):
    """Synthetic round of certificates in the reference's byte formats
    (SURVEY.md 8(d) C3/C1): committee keys seed_i = SHA512("coa-key"||i),
    header author = member c mod N with n_payload batch digests (worker 0)
    and the previous round's 2f+1 certificate digests as parents (shared by
    every header of the round, as in Narwhal), votes from n_votes distinct
    members rotated by certificate index (rotate=False: the same members in
    the same positions), all signed on the device."""
    import workloads

    N = committee_size
    seeds = workloads.key_seeds(N)
    pks = coa_crypto.public_keys(seeds)
    committee = Committee({bytes(p): 1 for p in pks}, {bytes(p): {0} for p in pks})
    q = committee.quorum_threshold()
    n_votes = n_votes or q
    rng = np.random.default_rng(seed)
    parents = sorted(bytes(x) for x in rng.integers(0, 256, (q, 32), dtype=np.uint8))
    author_idx = np.arange(n_certs) % N
    header_inputs = []
    for c in range(n_certs):
        pay = rng.integers(0, 256, (n_payload, 32), dtype=np.uint8)
        out = bytearray(bytes(pks[author_idx[c]])) + struct.pack("<Q", round_)
        for d in sorted(bytes(x) for x in pay):
            out += d + struct.pack("<I", 0)
        for p in parents:
            out += p
        header_inputs.append(bytes(out))
    ids = coa_crypto.sha512_many(header_inputs)[:, :32].copy()
    a_seeds = seeds[author_idx]
    _, hsigs = coa_crypto.sign_many(a_seeds, ids)
    authors = pks[author_idx].copy()
    cin = [bytes(ids[c]) + struct.pack("<Q", round_) + bytes(authors[c]) for c in range(n_certs)]
    cdg = coa_crypto.sha512_many(cin)[:, :32].copy()
    # rotate=False: vote position v is member v in every certificate
    voter_idx = ((np.arange(n_certs)[:, None] * int(rotate) + np.arange(n_votes)[None, :]) % N).reshape(-1)
    vmsgs = np.repeat(cdg, n_votes, axis=0)
    vpks, vsigs = coa_crypto.sign_many(seeds[voter_idx], vmsgs)
    offs = np.arange(0, n_certs * n_votes + 1, n_votes, dtype=np.uint64)
    return committee, CertificateBatch(header_inputs, ids, authors, hsigs, cdg, vpks, vsigs, offs, voter_idx,
                                       author_idx, round_)


def _quorum_errors(batch, committee):
    """Certificate::verify's vote checks (primary/src/messages.rs:196-211) over
    a CertificateBatch, read from the vote keys themselves (not from the
    synthetic voter_idx): a key outside the committee (stake 0,
    UnknownAuthority), a key voting twice (AuthorityReuse) or less than
    2N/3 + 1 of stake (CertificateRequiresQuorum) marks the certificate.
    Returns uint8 [n]: 1 = one of those errors."""
    n = len(batch)
    err = np.zeros(n, np.uint8)
    nv = int(batch.offsets[-1]) if n else 0
    if nv == 0:
        return np.ones(n, np.uint8) if committee.quorum_threshold() > 0 else err
    keys = np.ascontiguousarray(batch.vote_pks[:nv], dtype=np.uint8).view(np.dtype((np.void, 32))).reshape(-1)
    uniq, inv = np.unique(keys, return_inverse=True)
    ustake = np.array([committee.stake(PublicKey(bytes(u))) for u in uniq], np.int64)
    vstake = ustake[inv]
    q = committee.quorum_threshold()
    for i in range(n):
        lo, hi = int(batch.offsets[i]), int(batch.offsets[i + 1])
        k = inv[lo:hi]
        st = vstake[lo:hi]
        if (st <= 0).any() or len(np.unique(k)) != len(k) or int(st.sum()) < q:
            err[i] = 1
    return err


def verify_certificate_batch(batch, committee, rng_seed=0):
    """Certificate::verify over a CertificateBatch: one fused engine call
    (coa_certificate_verify_many) + vectorised protocol checks.
    Returns uint8 [n]: 0 Ok, 1 Err."""
    n = len(batch)
    rounds = np.full(n, batch.round, np.uint64)
    st = coa_crypto.certificate_verify_many(batch.header_inputs, batch.ids, batch.authors, batch.header_sigs, rounds,
                                            batch.vote_pks, batch.vote_sigs, batch.offsets, rng_seed=rng_seed)
    err = (st != 0).astype(np.uint8)
    stake = np.array([committee.stake(PublicKey(bytes(p))) for p in batch.authors])
    err |= (stake <= 0).astype(np.uint8)                                        # UnknownAuthority
    err |= _quorum_errors(batch, committee)                                     # votes: stake, reuse, quorum
    return err


def verify_certificate_batch_stepwise(batch, committee, rng_seed=0):
    """The same over the per-primitive entry points (four engine calls)."""
    n = len(batch)
    err = np.zeros(n, np.uint8)
    hd = coa_crypto.sha512_many(batch.header_inputs)[:, :32]
    err |= (hd != batch.ids).any(axis=1).astype(np.uint8)
    stake = np.array([committee.stake(PublicKey(bytes(p))) for p in batch.authors])
    err |= (stake <= 0).astype(np.uint8)
    err |= coa_crypto.verify_strict_many(batch.ids, batch.authors, batch.header_sigs)
    err |= _quorum_errors(batch, committee)
    cin = [bytes(batch.ids[c]) + struct.pack("<Q", batch.round) + bytes(batch.authors[c]) for c in range(n)]
    cd = coa_crypto.sha512_many(cin)[:, :32]
    gv = coa_crypto.verify_batch_groups(cd, batch.vote_pks, batch.vote_sigs, batch.offsets, rng_seed=rng_seed)
    return err | gv
