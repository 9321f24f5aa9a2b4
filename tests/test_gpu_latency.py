"""GPU: the single-signature latency route (coa_latency.hip k_verify_lat) --
Signature::verify one message at a time, as Header::verify / Vote::verify call
it (primary/src/messages.rs:64-66,139-141).  Calls of at most COA_LAT_MAX
(default 2,048) triples with 32-byte messages take it, on one idle context
(such calls are not sharded over GPUs); its verdicts must equal
the oracle's (dalek verify_strict) on the golden vectors and on adversarial
mixes, with the keys registered in the committee cache (comb path) and not
(halved-scalar row chains)."""
import os

import numpy as np
import pytest

import coa_oracle as co
from conftest import load_golden

pytestmark = pytest.mark.gpu


def _vec32():
    return [v for v in load_golden("verify_vectors.json") if len(v["msg"]) == 64]


@pytest.fixture
def no_committee(engine):
    engine.committee_register(np.zeros((0, 32), np.uint8))
    yield
    engine.committee_register(np.zeros((0, 32), np.uint8))


@pytest.mark.parametrize("cached", [False, True])
def test_golden_vectors_one_at_a_time(engine, no_committee, cached):
    vecs = _vec32()
    if cached:  # every key of the vectors, small-order and off-curve ones included
        engine.committee_register(np.array([list(bytes.fromhex(v["pk"])) for v in vecs], np.uint8))
    for v in vecs:
        sig = engine.Signature.from_bytes(bytes.fromhex(v["sig"]))
        try:
            sig.verify(bytes.fromhex(v["msg"]), bytes.fromhex(v["pk"]))
            got = True
        except engine.CryptoError:
            got = False
        assert got == v["expect"], (v["class"], v["note"], cached)


def _pool():
    return [(bytes.fromhex(v["msg"]), bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]))
            for v in load_golden("mixed_order_pool.json")]


@pytest.mark.parametrize("cached", [False, True])
@pytest.mark.parametrize("n,lat_max", [(64, None), (3000, "4096")])
def test_adversarial_mix_latency_route(engine, no_committee, monkeypatch, cached, n, lat_max):
    """n triples in one call routed to k_verify_lat (one workgroup each),
    25 % adversarial over the 8 classes, against the C oracle."""
    from workloads import adversarial_mix, key_seeds, messages

    if lat_max:
        monkeypatch.setenv("COA_LAT_MAX", lat_max)
    seeds, msgs = key_seeds(n, 300), messages(n, 300)
    pks, sigs = engine.sign_many(seeds, msgs)
    msgs, pks, sigs, cls = adversarial_mix(msgs, pks, sigs, frac=0.25, seed=n, mixed_pool=_pool())
    if cached:
        engine.committee_register(pks)
    got = engine.verify_strict_many(msgs, pks, sigs)
    exp = co.verify_strict_many(msgs, pks, sigs, min(16, os.cpu_count() or 1))
    mism = np.nonzero(got != exp)[0]
    assert mism.size == 0, [(int(i), int(cls[i])) for i in mism[:20]]
    assert (got[cls == 7] == 0).all() and (got[cls == -1] == 0).all()


def test_latency_route_matches_throughput_route(engine, no_committee, monkeypatch):
    """The same 64 triples through both routes (COA_LAT_MAX=0 forces the
    split throughput kernels)."""
    from workloads import adversarial_mix, key_seeds, messages

    n = 64
    pks, sigs = engine.sign_many(key_seeds(n, 900), messages(n, 900))
    msgs, pks, sigs, _ = adversarial_mix(messages(n, 900), pks, sigs, frac=0.5, seed=5, mixed_pool=_pool())
    a = engine.verify_strict_many(msgs, pks, sigs)
    monkeypatch.setenv("COA_LAT_MAX", "0")
    b = engine.verify_strict_many(msgs, pks, sigs)
    assert (a == b).all()
