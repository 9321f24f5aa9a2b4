"""GPU: engine-failure recovery, concurrency of the latency route and
registration under load.

* Host-pointer calls (coa_runtime.cpp for_shards): with COA_FAULT_SHARD a
  shard's work is declared failed after it ran; its context is rebuilt (new
  stream, per-call buffers released) and the shard re-run on the next
  context -- verdicts stay bit-exact against the C oracle and
  coa_engine_recoveries counts it.  The reference's verify never fails for a
  reason other than the input, and Core::run logs and continues
  (primary/src/core.rs:390-398), so a device hiccup must not become a verdict.
* One-message calls (Header::verify / Vote::verify,
  primary/src/messages.rs:64-66,139-141) from 8 threads over 8 contexts: each
  call takes an idle context (no longer always the first), every verdict
  equals the golden expectation.
* coa_committee_register while the aggregation queue is saturated with
  certificate windows: registration builds the next key-cache generation
  beside the current one and swaps it in, while every window keeps the
  generation it pinned at launch (coa_keycache_pin) -- no gate, so no window
  is held back (test_registration_never_holds_a_window_back: none above
  5 ms) and every certificate verdict stays exact whether the committee is
  registered, re-registered or cleared meanwhile."""
import os
import threading

import numpy as np
import pytest

import coa_oracle as co
from conftest import load_golden

pytestmark = pytest.mark.gpu


def _vec32():
    return [v for v in load_golden("verify_vectors.json") if len(v["msg"]) == 64]


def _tiled(n):
    vecs = _vec32()
    rows = [vecs[i % len(vecs)] for i in range(n)]
    msgs = np.array([list(bytes.fromhex(v["msg"])) for v in rows], np.uint8)
    pks = np.array([list(bytes.fromhex(v["pk"])) for v in rows], np.uint8)
    sigs = np.array([list(bytes.fromhex(v["sig"])) for v in rows], np.uint8)
    exp = np.array([0 if v["expect"] else 1 for v in rows], np.uint8)
    return msgs, pks, sigs, exp


@pytest.fixture
def contexts(engine):
    """Re-open the engine with k contexts on device 0 (k index-range shards,
    as k GPUs of a node); back to the default afterwards."""
    opened = []

    def open_k(k):
        engine.shutdown()
        engine.init_devices([0] * k)
        opened.append(k)
        return engine

    yield open_k
    if opened:
        engine.shutdown()
        engine.init(0)


@pytest.mark.parametrize("k", [1, 3])
def test_shard_failure_rebuilds_context_and_reruns(engine, contexts, monkeypatch, k):
    from workloads import adversarial_mix, key_seeds, messages

    contexts(k)
    n = 12_000  # above COA_LAT_MAX: the sharded throughput path
    pks, sigs = engine.sign_many(key_seeds(n, 7000), messages(n, 7000))
    msgs, pks, sigs, cls = adversarial_mix(messages(n, 7000), pks, sigs, frac=0.1, seed=77)
    exp = co.verify_strict_many(msgs, pks, sigs, min(16, os.cpu_count() or 1))
    before = engine.engine_recoveries()
    monkeypatch.setenv("COA_FAULT_SHARD", "2")  # every 2nd shard "fails"
    got = engine.verify_strict_many(msgs, pks, sigs)
    got2 = engine.verify_strict_many(msgs, pks, sigs)
    monkeypatch.delenv("COA_FAULT_SHARD")
    after = engine.engine_recoveries()
    assert (got == exp).all() and (got2 == exp).all()
    assert after["contexts_rebuilt"] > before["contexts_rebuilt"]
    assert after["shards_rerun"] > before["shards_rerun"]
    # the rebuilt contexts keep working: SHA-512 and the golden tiles
    m2, p2, s2, e2 = _tiled(5000)
    assert (engine.verify_strict_many(m2, p2, s2) == e2).all()


def test_every_context_failed_then_the_cpu_path_answers(engine, contexts, monkeypatch):
    """COA_FAULT_SHARD=all: every attempt on every context fails, so the GPU
    call itself fails loudly (EngineError, no silent fallback).  What the
    Rust binding then answers with (degrade.rs, COA_ON_ENGINE_FAILURE=cpu) is
    the engine's own CPU path, coa_cpu_*: its verdicts equal the GPU's
    fault-free verdicts and the oracle's, for signatures and certificates."""
    import certificates as C
    from workloads import adversarial_mix, key_seeds, messages

    contexts(2)
    n = 12_000
    pks, sigs = engine.sign_many(key_seeds(n, 8100), messages(n, 8100))
    msgs, pks, sigs, _ = adversarial_mix(messages(n, 8100), pks, sigs, frac=0.1, seed=78)
    gpu = engine.verify_strict_many(msgs, pks, sigs)
    # 600 certificates x 4 jobs: above the latency route (2,048 jobs), so the
    # call is sharded over the contexts (for_shards)
    committee, batch = C.synth_certificates(600, committee_size=4, n_payload=1, seed=5)
    bad = batch.vote_sigs.copy()
    bad[7, 40] ^= 1
    rounds = np.full(600, batch.round, np.uint64)
    cargs = (batch.header_inputs, batch.ids, batch.authors, batch.header_sigs, rounds, batch.vote_pks, bad,
             batch.offsets)
    gpu_c = engine.certificate_verify_many(*cargs)
    monkeypatch.setenv("COA_FAULT_SHARD", "all")
    with pytest.raises(engine.EngineError):
        engine.verify_strict_many(msgs, pks, sigs)
    with pytest.raises(engine.EngineError):
        engine.certificate_verify_many(*cargs)
    cpu = engine.cpu_verify_strict_many(msgs, pks, sigs)
    cpu_c = engine.cpu_certificate_verify_many(*cargs)
    monkeypatch.delenv("COA_FAULT_SHARD")
    exp = co.verify_strict_many(msgs, pks, sigs, min(16, os.cpu_count() or 1))
    assert (gpu == exp).all() and (cpu == exp).all()
    assert list(cpu_c) == list(gpu_c) and int(np.count_nonzero(gpu_c)) == 1
    # the contexts were rebuilt and answer again
    m2, p2, s2, e2 = _tiled(5000)
    assert (engine.verify_strict_many(m2, p2, s2) == e2).all()


def test_single_verifies_from_eight_threads_over_eight_contexts(engine, contexts):
    contexts(8)
    vecs = _vec32()
    engine.committee_register(np.array([list(bytes.fromhex(v["pk"])) for v in vecs[:40]], np.uint8))
    errors = []

    def worker(t):
        try:
            for r in range(3):
                for i in range(t, len(vecs), 8):
                    v = vecs[i]
                    sig = engine.Signature.from_bytes(bytes.fromhex(v["sig"]))
                    try:
                        sig.verify(bytes.fromhex(v["msg"]), bytes.fromhex(v["pk"]))
                        got = True
                    except engine.CryptoError:
                        got = False
                    if got != v["expect"]:
                        errors.append((t, r, v["class"], v["note"]))
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=240)
    engine.committee_register(np.zeros((0, 32), np.uint8))
    assert not any(x.is_alive() for x in th)
    assert not errors, errors[:10]


def test_register_while_queue_saturated_with_certificates(engine):
    import certificates as C

    committee, batch = C.synth_certificates(48, committee_size=12, n_payload=3, seed=31)
    batch.vote_sigs[int(batch.offsets[5]) + 1, 44] ^= 1   # certificate 5: bad vote
    batch.header_sigs[9, 20] ^= 1                          # certificate 9: bad header signature
    committee.register()
    want_bits = {5: engine.CERT_BAD_VOTES, 9: engine.CERT_BAD_HEADER_SIG}
    stop = threading.Event()
    regs = [0]

    def registrar():
        while not stop.is_set():
            engine.committee_register(np.zeros((0, 32), np.uint8))   # cleared: uncached host path
            committee.register()                                      # back: cached fused kernel
            regs[0] += 1

    results = []
    lock = threading.Lock()
    with engine.AggregationQueue(max_batch=512, max_delay_us=300) as q:
        def producer(t):
            out = []
            for rnd in range(6):
                for c in range(t, len(batch), 4):
                    lo, hi = int(batch.offsets[c]), int(batch.offsets[c + 1])
                    votes = [(engine.PublicKey(bytes(batch.vote_pks[j])),
                              engine.Signature.from_bytes(bytes(batch.vote_sigs[j]))) for j in range(lo, hi)]
                    out.append((c, q.submit_certificate(batch.header_inputs[c], bytes(batch.ids[c]),
                                                        bytes(batch.authors[c]), bytes(batch.header_sigs[c]),
                                                        batch.round, votes)))
            with lock:
                results.extend(out)

        reg = threading.Thread(target=registrar)
        reg.start()
        th = [threading.Thread(target=producer, args=(t,)) for t in range(4)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        q.flush()
        stop.set()
        reg.join()
        for c, f in results:
            assert f.result(timeout=120) == want_bits.get(c, 0), c
        m = q.metrics()
    committee.register()
    assert regs[0] >= 1 and m["certificates"] == len(results) and m["failed_windows"] == 0


def test_registration_never_holds_a_window_back(engine, monkeypatch):
    """coa_committee_register builds the next key-cache
    generation beside the current one (on a least-priority stream) and swaps
    it in; windows in flight keep the generation they pinned.
    A committee-100 re-registration (65 GB of radix-2^20 combs, ~0.6 s),
    twice, under a steady certificate stream of 5,000 certificates/s: every
    verdict exact, and no window takes longer than 5 ms from its launch call
    to its outputs (round 3's write gate held windows back for the whole
    0.6-2.7 s build).

    The stream is submitted and answered in C (tools/latc.c latc_paced, idle
    launch as a node's PreVerifier runs it): a window's time then contains
    only the engine.  Through Python callbacks it also contained the
    interpreter -- a generation-2 collection (27-89 ms, round 5:
    profiles/r05_register_gc.txt) or any other pause of the thread holding
    the GIL stalls the completion thread, and round 6 saw a 338 ms window
    that way with collection off and every engine stage of the trace short."""
    import time

    import bench
    import certificates as C

    committee, batch = C.synth_certificates(64, committee_size=100, n_payload=4, seed=41)
    batch.header_sigs[7, 20] ^= 1                          # certificate 7: bad header signature
    cexp = np.zeros(len(batch), np.uint8)
    cexp[7] = engine.CERT_BAD_HEADER_SIG
    committee.register()
    reg_s, t_reg = [], []

    def registrar():
        time.sleep(0.4)
        for _ in range(2):
            t0 = time.perf_counter()
            committee.register()
            reg_s.append(time.perf_counter() - t0)
            t_reg.append((t0, time.perf_counter()))

    monkeypatch.setenv("COA_QUEUE_IDLE_LAUNCH", "1")  # read at queue creation (latc_paced creates its queue)
    n = 12_000  # 2.4 s at 5,000 certificates/s: both registrations fall inside
    arrive = np.arange(n, dtype=np.float64) / 5000.0
    reg = threading.Thread(target=registrar)
    t_stream = time.perf_counter()
    reg.start()
    # paced_queue asserts that every answer equals its expectation
    lat, el, met = bench.paced_queue(arrive, np.ones(n, np.int32), np.arange(n, dtype=np.uint32) % len(batch),
                                     certs=batch, cexp=cexp, max_batch=4096, max_delay_us=200)
    t_end = time.perf_counter()
    reg.join(timeout=60)
    assert not reg.is_alive() and len(reg_s) == 2, reg_s
    assert all(t_stream < a and b < t_end for a, b in t_reg), (t_stream, t_reg, t_end)  # built under the stream
    assert met["failed_windows"] == 0 and met["certificates"] == n
    assert met["window_us_max"] < 5000, (met["window_us_max"], met["window_max_items"], met["window_max_device_us"],
                                         reg_s)


def test_failed_windows_retried_while_registering(engine, monkeypatch):
    """a window whose launch fails is re-run on the recovery
    context by the completer while coa_committee_register runs.  With round
    3's key-cache gate that could deadlock (the retry waiting for readers only
    the completer could release); with generation pins the retry takes the
    current generation and nothing waits.  Every 3rd window fails
    (COA_QUEUE_FAULT, read at queue creation) while a registrar alternates
    clear / register; every verdict exact, every failed window recovered."""
    import certificates as C

    monkeypatch.setenv("COA_QUEUE_FAULT", "3")
    committee, batch = C.synth_certificates(48, committee_size=12, n_payload=3, seed=37)
    batch.vote_sigs[int(batch.offsets[4]) + 2, 40] ^= 1   # certificate 4: bad vote
    want = {4: engine.CERT_BAD_VOTES}
    committee.register()
    stop = threading.Event()
    regs = [0]

    def registrar():
        while not stop.is_set():
            engine.committee_register(np.zeros((0, 32), np.uint8))
            committee.register()
            regs[0] += 1

    results = []
    lock = threading.Lock()
    with engine.AggregationQueue(max_batch=256, max_delay_us=200) as q:
        def producer(t):
            out = []
            for rnd in range(5):
                for c in range(t, len(batch), 2):
                    lo, hi = int(batch.offsets[c]), int(batch.offsets[c + 1])
                    votes = [(engine.PublicKey(bytes(batch.vote_pks[j])),
                              engine.Signature.from_bytes(bytes(batch.vote_sigs[j]))) for j in range(lo, hi)]
                    out.append((c, q.submit_certificate(batch.header_inputs[c], bytes(batch.ids[c]),
                                                        bytes(batch.authors[c]), bytes(batch.header_sigs[c]),
                                                        batch.round, votes)))
            with lock:
                results.extend(out)

        reg = threading.Thread(target=registrar)
        reg.start()
        th = [threading.Thread(target=producer, args=(t,)) for t in range(2)]
        for x in th:
            x.start()
        for x in th:
            x.join(timeout=180)
        q.flush()
        stop.set()
        reg.join(timeout=180)
        assert not reg.is_alive() and not any(x.is_alive() for x in th)
        for c, f in results:
            assert f.result(timeout=120) == want.get(c, 0), c
        m = q.metrics()
    committee.register()
    assert regs[0] >= 1 and m["certificates"] == len(results)
    assert m["retried_windows"] >= 1 and m["recovered_windows"] == m["retried_windows"] and m["failed_windows"] == 0, m
