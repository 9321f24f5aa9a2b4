"""GPU: the exact decision of certificates the fused kernel leaves open
(coa_runtime.cpp resolve_raw / cert_resolve; the aggregation queue's resolver
reaches it through coa_certificate_resolve_raw).

A small round (committee 10, registered) with certificates whose author or
one voter is outside the committee, each with and without a failing check,
through coa_certificate_verify_many -- small enough (votes + headers <= 2,048)
for the one-launch exact path (a latency launch carrying the votes as the
verify_batch prefilter and the header signatures as plain verify_strict,
LatArgs::batch_n), and again with that path off (COA_RESOLVE_ONE_LAUNCH=0:
the prefilter launch, then the header launch).  Both give the C oracle's
bits, check by check (oracle/coa_oracle.c: Header::digest == id,
Signature::verify(id, author), verify_batch(Certificate::digest, votes) --
primary/src/messages.rs:48-84,189-234)."""
import os
import struct

import numpy as np
import pytest

import coa_oracle as co

pytestmark = pytest.mark.gpu

SMALL_ORDER_R = bytes.fromhex("c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a")


def _round(engine):
    import certificates as C
    import workloads

    n, size = 14, 10
    committee, b = C.synth_certificates(n, committee_size=size, n_payload=3, seed=77)
    committee.register()
    hin = list(b.header_inputs)
    ids, authors, hsigs = b.ids.copy(), b.authors.copy(), b.header_sigs.copy()
    vpks, vsigs = b.vote_pks.copy(), b.vote_sigs.copy()
    nv = int(b.offsets[1] - b.offsets[0])

    def reauthor(c, seed_start):
        """certificate c re-authored by a key outside the committee, every
        signature valid (votes by committee keys over the new digest)"""
        seed = workloads.key_seeds(1, start=seed_start)
        apk = engine.public_keys(seed)[0]
        h = bytes(apk) + hin[c][32:]
        hin[c] = h
        ids[c] = engine.sha512_many([h])[0, :32]
        authors[c] = apk
        _, hs = engine.sign_many(seed, ids[c:c + 1])
        hsigs[c] = hs[0]
        cd = engine.sha512_many([bytes(ids[c]) + struct.pack("<Q", b.round) + bytes(apk)])[0, :32]
        lo = int(b.offsets[c])
        vseeds = workloads.key_seeds(size)[(c + np.arange(nv)) % size]
        p, s = engine.sign_many(vseeds, np.tile(cd, (nv, 1)))
        vpks[lo:lo + nv], vsigs[lo:lo + nv] = p, s

    def foreign_vote(c, seed_start):
        """one vote of certificate c by a key outside the committee, valid"""
        v = int(b.offsets[c]) + 1
        p, s = engine.sign_many(workloads.key_seeds(1, start=seed_start), b.cert_digests[c:c + 1])
        vpks[v], vsigs[v] = p[0], s[0]
        return v

    reauthor(0, 900_000)                      # author outside: Ok
    reauthor(1, 900_100)
    hsigs[1, 40] ^= 1                         # author outside, bad header signature
    reauthor(2, 900_200)
    vsigs[int(b.offsets[2]) + 2, 50] ^= 1     # author outside, a bad vote
    foreign_vote(3, 900_300)                  # a voter outside: Ok
    v = foreign_vote(4, 900_400)
    vsigs[v, 45] ^= 1                         # a voter outside, its own vote bad
    foreign_vote(5, 900_500)
    vsigs[int(b.offsets[5]) + 3, :32] = np.frombuffer(SMALL_ORDER_R, np.uint8)  # ... and a small-order R
    reauthor(6, 900_600)
    h = bytearray(hin[6]); h[60] ^= 1; hin[6] = bytes(h)  # author outside, header bytes changed: bad id
    foreign_vote(7, 900_700)
    hsigs[7, 33] ^= 1                         # a voter outside, bad header signature (author cached)
    vsigs[int(b.offsets[8]) + 1, 44] ^= 1     # cached keys, a bad vote (inconclusive -> exact)
    return b, hin, ids, authors, hsigs, vpks, vsigs


@pytest.mark.parametrize("one_launch", ["1", "0"])
def test_open_certificates_exact_against_oracle(engine, monkeypatch, one_launch):
    b, hin, ids, authors, hsigs, vpks, vsigs = _round(engine)
    monkeypatch.setenv("COA_RESOLVE_ONE_LAUNCH", one_launch)
    got = engine.certificate_verify_many(hin, ids, authors, hsigs, np.full(len(hin), b.round, np.uint64), vpks,
                                         vsigs, b.offsets)
    zs = np.random.default_rng(5).integers(0, 256, (int(b.offsets[-1]), 16), dtype=np.uint8)
    exp = co.certificate_verify_many(hin, ids, authors, hsigs, b.round, vpks, vsigs, b.offsets, zs,
                                     min(8, os.cpu_count() or 1))
    assert list(got) == list(exp)
    want = {0: 0, 1: 2, 2: 4, 3: 0, 4: 4, 5: 4, 6: 1, 7: 2, 8: 4}
    for c, bits in want.items():
        assert got[c] == bits, (c, int(got[c]))
    assert (got[9:] == 0).all()
