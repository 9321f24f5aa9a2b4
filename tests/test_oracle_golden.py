"""CPU: the oracle (oracle/ed25519_ref.py, dalek 1.0.1 semantics) reproduces
every committed golden fixture.  The fixtures were cross-checked against
libsodium 1.0.18 and the reference's own test fixtures when generated
(tests/golden/make_golden.py), so this pins the oracle on a machine without
libsodium too."""
import hashlib

import pytest

import ed25519_ref as o
from conftest import load_golden


def test_reference_fixtures():
    ref = load_golden("reference_crypto.json")
    seeds = [bytes.fromhex(s) for s in ref["seeds"]]
    pks = [bytes.fromhex(p) for p in ref["public_keys"]]
    # keys(): StdRng::from_seed([0;32]) + generate_keypair (crypto_tests.rs:26-29)
    assert [o.public_key(s) for s in seeds] == pks
    hello = bytes.fromhex(ref["hello_digest"])
    assert o.digest32(b"Hello, world!") == hello
    sig = bytes.fromhex(ref["hello_sig_key3"])
    assert o.sign(seeds[3], hello) == sig
    assert o.verify_strict(hello, pks[3], sig)  # verify_valid_signature
    assert not o.verify_strict(bytes.fromhex(ref["bad_digest"]), pks[3], sig)  # verify_invalid_signature
    zs = [int(z, 16) for z in ref["batch_zs"]]
    for key, expect in (("batch_valid", True), ("batch_invalid", False)):
        votes = [(bytes.fromhex(p), bytes.fromhex(s)) for p, s in ref[key]]
        assert o.verify_batch(hello, [p for p, _ in votes], [s for _, s in votes], zs) is expect
    ser = bytes.fromhex(ref["serialized_batch"])
    assert o.digest32(ser).hex() == ref["batch_digest"]  # worker batch_digest()


def test_verify_vectors():
    vecs = load_golden("verify_vectors.json")
    assert len(vecs) > 200
    for v in vecs:
        got = o.verify_strict(bytes.fromhex(v["msg"]), bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]))
        assert got == v["expect"], (v["class"], v["note"])


def test_batch_vectors():
    for g in load_golden("batch_vectors.json"):
        got = o.verify_batch(bytes.fromhex(g["msg"]), [bytes.fromhex(p) for p in g["pks"]],
                             [bytes.fromhex(s) for s in g["sigs"]], [int(z, 16) for z in g["zs"]])
        assert got == g["expect"], g["name"]


def test_sha512_vectors():
    for v in load_golden("sha512_vectors.json"):
        assert hashlib.sha512(bytes.fromhex(v["msg"])).hexdigest() == v["sha512"]


def test_small_order_encodings_complete():
    enc = o.small_order_encodings()
    assert len(enc) == 14  # 8 torsion points, both signs where decodable, y >= p forms
    for e in enc:
        assert o.is_small_order(o.decompress(e))


@pytest.mark.parametrize("y", [2, 3, 5, 7])
def test_noncanonical_y_is_accepted_by_decompress(y):
    # dalek's FieldElement::from_bytes keeps y in [p, 2^255): y + p decodes like y
    a = o.decompress(y.to_bytes(32, "little"))
    b = o.decompress((y + o.P).to_bytes(32, "little"))
    assert (a is None) == (b is None)
    if a is not None:
        assert o.peq(a, b)
