"""GPU: the reference's verify callers (primary/src/messages.rs:48-234) over
the engine -- Header/Vote/Certificate::verify check order, error kinds and
the batched path agree with the oracle-checked crypto (mirrors
primary/src/tests/core_tests.rs process_header / process_votes /
process_certificates)."""
import numpy as np
import pytest

import coa_oracle as co
import ed25519_ref as o

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def round_c1(engine):
    import certificates as C

    return C.synth_certificates(6, committee_size=4, n_payload=2, seed=1)


@pytest.fixture(scope="module")
def round_c3(engine):
    import certificates as C

    return C.synth_certificates(40, committee_size=100, n_payload=32, seed=2)


def test_c1_certificates_verify(round_c1):
    import certificates as C

    committee, batch = round_c1
    assert committee.quorum_threshold() == 3
    for i in range(len(batch)):
        cert = batch.certificate(i)
        assert len(cert.votes) == 3
        cert.verify(committee, rng_seed=5)
        # the vote crypto equals the oracle's per-signature verdicts
        d = bytes(batch.cert_digests[i])
        for pk, sg in cert.votes:
            assert co.verify_strict(d, bytes(pk), sg.flatten())
    assert (C.verify_certificate_batch(batch, committee) == 0).all()


def test_c3_shape_and_batch(round_c3):
    import certificates as C

    committee, batch = round_c3
    assert committee.quorum_threshold() == 67
    assert all(len(h) == 3336 for h in batch.header_inputs)  # 32 payload + 67 parents
    assert int(batch.offsets[1]) == 67
    assert (C.verify_certificate_batch(batch, committee, rng_seed=9) == 0).all()


def test_certificate_error_kinds(round_c3, engine):
    import certificates as C

    committee, batch = round_c3
    good = batch.certificate(0)
    good.verify(committee)
    # InvalidSignature: one corrupted vote
    bad = batch.certificate(1)
    sg = bytearray(bad.votes[10][1].flatten()); sg[40] ^= 1
    bad.votes[10] = (bad.votes[10][0], engine.Signature.from_bytes(bytes(sg)))
    with pytest.raises(C.InvalidSignature):
        bad.verify(committee)
    # AuthorityReuse
    bad = batch.certificate(2)
    bad.votes[5] = bad.votes[4]
    with pytest.raises(C.AuthorityReuse):
        bad.verify(committee)
    # CertificateRequiresQuorum
    bad = batch.certificate(3)
    bad.votes = bad.votes[:66]
    with pytest.raises(C.CertificateRequiresQuorum):
        bad.verify(committee)
    # UnknownAuthority (voter outside the committee)
    bad = batch.certificate(4)
    bad.votes[0] = (engine.PublicKey(bytes(32)), bad.votes[0][1])
    with pytest.raises(C.UnknownAuthority):
        bad.verify(committee)
    # InvalidHeaderId
    bad = batch.certificate(5)
    bad.header._digest_input = bad.header._digest_input[:-1] + b"\x00"
    with pytest.raises(C.InvalidHeaderId):
        bad.verify(committee)
    # header signature by the wrong key
    bad = batch.certificate(6)
    bad.header.signature = batch.certificate(7).header.signature
    with pytest.raises(C.InvalidSignature):
        bad.verify(committee)
    # genesis certificates verify without crypto
    g = C.Certificate(C.Header(author=committee.authorities()[0]), [])
    g.verify(committee)
    # the batched path returns the same Ok/Err pattern
    certs = [batch.certificate(i) for i in range(8)]
    certs[1].votes[3] = (certs[1].votes[3][0], engine.Signature())
    certs[4].votes = certs[4].votes[:10]
    res = C.verify_certificates(certs + [g], committee)
    assert [type(r).__name__ if r else None for r in res] == [
        None, "InvalidSignature", None, None, "CertificateRequiresQuorum", None, None, None, None]


def test_vote_verify(round_c1, engine):
    import certificates as C

    committee, batch = round_c1
    cert = batch.certificate(0)
    pk, sg = cert.votes[1]
    v = C.Vote(cert.header.id, batch.round, cert.origin(), pk, sg)
    assert v.digest() == engine.Digest(bytes(batch.cert_digests[0]))  # Vote::digest == Certificate::digest
    v.verify(committee)
    v.author = cert.votes[2][0]
    with pytest.raises(C.InvalidSignature):
        v.verify(committee)
