"""Wire decode of PrimaryMessage frames (coa_wire.cpp).

CPU: frames built by an independent encoder (tests/wire_codec.py, from the
reference's serde derives) decode to exactly the fields and the
Header::digest input the reference hashes (BTreeMap/BTreeSet order, last
value of a repeated payload key); truncation at every byte, unknown
variants, malformed base64 keys and over-long keys behave as bincode 1.3 +
PublicKey::decode_base64 do (a key decoding to < 32 bytes panics in the
reference, crypto/src/lib.rs:74, and is an error here).  Non-canonical base64
acceptance follows base64 0.13's rules and is parity unpinned (the crate is
not available in this image).
GPU: a C3 round serialised to frames, decoded and verified by one
coa_certificate_verify_many call."""
import base64
import random

import numpy as np
import pytest

import wire_codec as W


def _rand(rng, n):
    return bytes(rng.getrandbits(8) for _ in range(n))


def _lib():
    import build

    build.build()
    import coa_crypto

    return coa_crypto


def _cert(rng, n_payload=5, n_parents=4, n_votes=3, dup=False):
    author = _rand(rng, 32)
    payload = [(_rand(rng, 32), rng.getrandbits(32)) for _ in range(n_payload)]
    if dup and payload:
        payload.append((payload[0][0], 77))  # repeated key: the later value wins
    parents = [_rand(rng, 32) for _ in range(n_parents)]
    if dup and parents:
        parents.append(parents[-1])
    id_, sig = _rand(rng, 32), _rand(rng, 64)
    rnd = rng.getrandbits(64)
    votes = [(_rand(rng, 32), _rand(rng, 64)) for _ in range(n_votes)]
    hb = W.header(author, rnd, payload, parents, id_, sig)
    frame = W.primary_message(2, W.certificate(hb, votes))
    return frame, dict(author=author, round=rnd, payload=payload, parents=parents, id=id_, sig=sig, votes=votes)


def test_certificate_frames_roundtrip():
    cc = _lib()
    rng = random.Random(1)
    frames, want = [], []
    for i in range(40):
        f, w = _cert(rng, n_payload=i % 7, n_parents=(3 * i) % 5, n_votes=i % 9, dup=i % 3 == 0)
        frames.append(f)
        want.append(w)
    kinds, hb, nv = cc.wire_scan(frames)
    assert (kinds == cc.MSG_CERTIFICATE).all()
    d = cc.wire_decode_certificates(frames)
    for i, w in enumerate(want):
        exp_in = W.header_digest_input(w["author"], w["round"], w["payload"], w["parents"])
        assert d["header_inputs"][i] == exp_in and int(hb[i]) == len(exp_in)
        assert bytes(d["ids"][i]) == w["id"] and bytes(d["origins"][i]) == w["author"]
        assert bytes(d["header_sigs"][i]) == w["sig"] and int(d["rounds"][i]) == w["round"]
        assert int(d["payload_counts"][i]) == len({bytes(p) for p, _ in w["payload"]})
        lo, hi = int(d["vote_offsets"][i]), int(d["vote_offsets"][i + 1])
        assert hi - lo == len(w["votes"]) == int(nv[i])
        for j, (pk, sg) in enumerate(w["votes"]):
            assert bytes(d["vote_pks"][lo + j]) == pk and bytes(d["vote_sigs"][lo + j]) == sg


def test_header_vote_request_frames():
    cc = _lib()
    rng = random.Random(2)
    a, o, i_, s = _rand(rng, 32), _rand(rng, 32), _rand(rng, 32), _rand(rng, 64)
    pay = [(_rand(rng, 32), 3), (_rand(rng, 32), 1)]
    par = [_rand(rng, 32)]
    hf = W.primary_message(0, W.header(a, 9, pay, par, i_, s))
    vf = W.primary_message(1, W.vote(i_, 9, o, a, s))
    rf = W.primary_message(3, W.cert_request([_rand(rng, 32)] * 3, a))
    kinds, _, _ = cc.wire_scan([hf, vf, rf])
    assert list(kinds) == [cc.MSG_HEADER, cc.MSG_VOTE, cc.MSG_CERT_REQUEST]
    h = cc.wire_decode_headers([hf])
    assert h["header_inputs"][0] == W.header_digest_input(a, 9, pay, par) and int(h["payload_counts"][0]) == 2
    assert bytes(h["ids"][0]) == i_ and bytes(h["authors"][0]) == a and bytes(h["sigs"][0]) == s
    v = cc.wire_decode_votes([vf])
    assert bytes(v["ids"][0]) == i_ and int(v["rounds"][0]) == 9
    assert bytes(v["origins"][0]) == o and bytes(v["authors"][0]) == a and bytes(v["sigs"][0]) == s
    with pytest.raises(cc.EngineError):
        cc.wire_decode_votes([hf])  # a Header frame is not a Vote


def test_truncation_and_malformed_keys():
    cc = _lib()
    rng = random.Random(3)
    f, w = _cert(rng, n_payload=2, n_parents=2, n_votes=2)
    # every strict prefix is an error (bincode reads fields in order; trailing bytes are allowed)
    kinds, _, _ = cc.wire_scan([f[:k] for k in range(len(f))])
    assert (kinds < 0).all()
    kinds, _, _ = cc.wire_scan([f + b"trailing"])
    assert kinds[0] == cc.MSG_CERTIFICATE
    # unknown enum variant
    assert cc.wire_scan([b"\x07\x00\x00\x00" + f[4:]])[0][0] == cc.WIRE_EFORMAT
    body = lambda field: W.primary_message(0, W.header(None, 1, [], [], bytes(32), bytes(64),  # noqa: E731
                                                       author_field=field))
    k32 = bytes(range(32))
    cases = {
        "canonical": (W.raw_key(base64.b64encode(k32)), k32),
        "unpadded": (W.raw_key(base64.b64encode(k32).rstrip(b"=")), k32),
        "longer key, first 32 bytes kept": (W.raw_key(base64.b64encode(k32 + b"tail!!")), k32),
        "short key (reference panics)": (W.raw_key(base64.b64encode(k32[:16])), None),
        "invalid character": (W.raw_key(base64.b64encode(k32)[:-3] + b"*A="), None),
        "non-zero trailing bits": (W.raw_key(base64.b64encode(k32)[:-2] + b"B="), None),
        "too much padding": (W.raw_key(base64.b64encode(k32) + b"=="), None),
        "not UTF-8": (W.raw_key(b"\xff" * 44), None),
    }
    for name, (field, expect) in cases.items():
        fr = body(field)
        kind = cc.wire_scan([fr])[0][0]
        if expect is None:
            assert kind < 0, name
        else:
            assert kind == cc.MSG_HEADER, name
            assert bytes(cc.wire_decode_headers([fr])["authors"][0]) == expect, name
    # a length prefix larger than the frame
    assert cc.wire_scan([body(b"\xff" * 8 + b"AAAA")])[0][0] == cc.WIRE_ETRUNC


@pytest.mark.gpu
def test_c3_frames_decode_and_verify(engine):
    import certificates as C

    committee, batch = C.synth_certificates(16, committee_size=100, n_payload=32, seed=8)
    committee.register()
    frames = []
    for i in range(len(batch)):
        hi_ = batch.header_inputs[i]
        # rebuild the header's payload/parents from its digest input (32 payload, 67 parents)
        pay = [(hi_[40 + 36 * k:72 + 36 * k], int.from_bytes(hi_[72 + 36 * k:76 + 36 * k], "little"))
               for k in range(32)]
        par = [hi_[40 + 36 * 32 + 32 * k:40 + 36 * 32 + 32 * (k + 1)] for k in range(67)]
        lo, hi = int(batch.offsets[i]), int(batch.offsets[i + 1])
        votes = [(bytes(batch.vote_pks[j]), bytes(batch.vote_sigs[j])) for j in range(lo, hi)]
        hb = W.header(bytes(batch.authors[i]), batch.round, pay[::-1], par[::-1], bytes(batch.ids[i]),
                      bytes(batch.header_sigs[i]))  # wire order reversed: the decoder re-sorts
        frames.append(W.primary_message(2, W.certificate(hb, votes)))
    frames[3] = frames[3][:-40] + bytes([frames[3][-40] ^ 1]) + frames[3][-39:]  # corrupt the last vote's R
    d = engine.wire_decode_certificates(frames)
    assert d["header_inputs"] == batch.header_inputs
    st = engine.certificate_verify_many(d["header_inputs"], d["ids"], d["origins"], d["header_sigs"], d["rounds"],
                                        d["vote_pks"], d["vote_sigs"], d["vote_offsets"], rng_seed=2)
    assert list(np.nonzero(st)[0]) == [3] and st[3] == engine.CERT_BAD_VOTES
