"""GPU: the primary's message pre-processing (Core::sanitize_*,
primary/src/core.rs:306-346) and the worker's Processor
(worker/src/processor.rs:35-55) over the engine.

A window of bincode PrimaryMessage frames (tests/wire_codec.py encoder) with
good and bad headers, votes and certificates goes through
Core.sanitize_frames -- native decode, one fused certificate launch, one
verify_strict launch per kind -- and every frame's result equals the
one-message-at-a-time path (Core.sanitize_* over objects), which follows the
reference's check order.  The Processor mirrors the reference's own
hash_and_store test (worker/src/tests/processor_tests.rs) on its golden
serialized batch."""
import hashlib
import struct

import numpy as np
import pytest

import wire_codec as W
from conftest import load_golden

pytestmark = pytest.mark.gpu


def _kind(e):
    return None if e is None else type(e).__name__


@pytest.fixture(scope="module")
def world(engine):
    import certificates as C

    committee, batch = C.synth_certificates(8, committee_size=4, n_payload=2, round_=5, seed=31)
    committee.register()
    return committee, batch


def _sign(engine, seed, msg):
    _, s = engine.sign_many(np.array([list(seed)], np.uint8), np.array([list(msg)], np.uint8))
    return bytes(s[0])


def test_sanitize_frames_matches_per_message_path(engine, world):
    import certificates as C
    import sanitize as S
    import workloads

    committee, batch = world
    seeds = workloads.key_seeds(4)
    pks = [bytes(p) for p in engine.public_keys(seeds)]
    frames, objs = [], []
    # certificates: valid, TooOld, bad vote, genesis
    for i in range(4):
        cert = batch.certificate(i)
        if i == 2:
            pk, sg = cert.votes[1]
            b = bytearray(sg.flatten())
            b[50] ^= 1
            cert.votes[1] = (pk, engine.Signature.from_bytes(bytes(b)))
        hi = cert.header.digest_input()
        pay = [(hi[40 + 36 * k:72 + 36 * k], struct.unpack_from("<I", hi, 72 + 36 * k)[0]) for k in range(2)]
        par = [hi[112 + 32 * k:144 + 32 * k] for k in range((len(hi) - 112) // 32)]
        rnd = 1 if i == 1 else batch.round  # TooOld when gc_round = 3 (round/gc checks run first)
        cert.header.round = rnd
        hb = W.header(bytes(cert.header.author), rnd, pay, par, bytes(cert.header.id),
                      cert.header.signature.flatten())
        frames.append(W.primary_message(2, W.certificate(hb, [(bytes(p), s.flatten()) for p, s in cert.votes])))
        cert.header.payload = {engine.Digest(d): w for d, w in pay}
        cert.header.parents = {engine.Digest(p) for p in par}
        cert.header._digest_input = None
        objs.append(("c", cert))
    g = C.Certificate(C.Header(author=committee.authorities()[0]), [])
    frames.append(W.primary_message(2, W.certificate(W.header(bytes(g.header.author), 0, [], [], bytes(32),
                                                              bytes(64)), [])))
    objs.append(("c", g))
    # headers: valid, wrong signer, worker id not in the committee
    for i, variant in enumerate(("ok", "bad_sig", "bad_worker")):
        a = i % 4
        pay = [(hashlib.sha512(b"batch%d" % i).digest()[:32], 7 if variant == "bad_worker" else 0)]
        par = [hashlib.sha512(b"parent%d" % i).digest()[:32]]
        hdr = C.Header(engine.PublicKey(pks[a]), 5, {engine.Digest(pay[0][0]): pay[0][1]},
                       {engine.Digest(par[0])})
        hdr.id = engine.Digest(hashlib.sha512(hdr.digest_input()).digest()[:32])
        signer = seeds[(a + 1) % 4] if variant == "bad_sig" else seeds[a]
        hdr.signature = engine.Signature.from_bytes(_sign(engine, signer, bytes(hdr.id)))
        frames.append(W.primary_message(0, W.header(pks[a], 5, pay, par, bytes(hdr.id), hdr.signature.flatten())))
        objs.append(("h", hdr))
    # votes on the current header: valid, unexpected, bad signature, unknown voter
    cur = objs[-3][1]
    for i, variant in enumerate(("ok", "unexpected", "bad_sig", "unknown")):
        v_id = bytes(cur.id) if variant != "unexpected" else bytes(32)
        vin = v_id + struct.pack("<Q", 5) + bytes(cur.author)
        vd = hashlib.sha512(vin).digest()[:32]
        voter = seeds[i % 4]
        author = pks[i % 4] if variant != "unknown" else bytes(engine.public_keys(np.array([[9] * 32], np.uint8))[0])
        sig = _sign(engine, voter if variant != "bad_sig" else seeds[(i + 1) % 4], vd)
        if variant == "unknown":
            sig = _sign(engine, bytes([9] * 32), vd)
        vote = C.Vote(engine.Digest(v_id), 5, cur.author, engine.PublicKey(author), engine.Signature.from_bytes(sig))
        frames.append(W.primary_message(1, W.vote(v_id, 5, bytes(cur.author), author, sig)))
        objs.append(("v", vote))
    # a certificates request and an undecodable frame
    frames.append(W.primary_message(3, W.cert_request([bytes(32)], pks[0])))
    frames.append(b"\x02\x00\x00\x00garbage")

    core = S.Core(committee, gc_round=3, current_header=cur)
    got = core.sanitize_frames(frames, rng_seed=4)
    want = []
    for kind, o in objs:
        try:
            {"c": core.sanitize_certificate, "h": core.sanitize_header, "v": core.sanitize_vote}[kind](o)
            want.append(None)
        except C.DagError as e:
            want.append(type(e).__name__)
    assert [_kind(e) for _, e in got[:len(objs)]] == want
    # the gc-round check precedes Certificate::verify's genesis exemption (core.rs:338-346)
    assert want == [None, "TooOld", "InvalidSignature", None, "TooOld", None, "InvalidSignature", "MalformedHeader",
                    None, "UnexpectedVote", "InvalidSignature", "UnknownAuthority"]
    assert got[-2] == (engine.MSG_CERT_REQUEST, None)
    # with gc_round 0 the genesis certificate is accepted without crypto
    assert S.Core(committee, gc_round=0, current_header=cur).sanitize_frames([frames[4]])[0][1] is None
    assert got[-1][0] is None and _kind(got[-1][1]) == "SerializationError"


def test_processor_hash_and_store(engine):
    """worker/src/tests/processor_tests.rs::hash_and_store on the reference's
    serialized batch (golden batch_digest 24d00f74...)."""
    import sanitize as S

    g = load_golden("reference_crypto.json")
    serialized = bytes.fromhex(g["serialized_batch"])
    digest = bytes.fromhex(g["batch_digest"])
    store = {}
    out = S.Processor(0, store, own_digest=True).process([serialized])
    assert out == [struct.pack("<I", 0) + digest + struct.pack("<I", 0)]  # bincode(OurBatch(digest, 0))
    assert store[digest] == serialized
    out = S.Processor(3, {}, own_digest=False).process([serialized, b"", serialized[:100]])
    assert out[0] == struct.pack("<I", 1) + digest + struct.pack("<I", 3)
    assert out[1][4:36] == hashlib.sha512(b"").digest()[:32]
