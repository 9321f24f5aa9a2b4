"""The native aggregation queue (coa_queue_*).

CPU part: coalescing, flush/destroy semantics and per-request callbacks from
many producer threads -- with no GPU every launch reports COA_ENODEVICE to
every request (no CPU fallback).  GPU part: verdicts through the queue equal
the oracle's."""
import threading

import numpy as np
import pytest

from conftest import load_golden


def _lib_built():
    import build

    build.build()
    import coa_crypto

    return coa_crypto


def test_queue_coalesces_and_reports_engine_errors_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by test_queue_verdicts_gpu")
    cc = _lib_built()
    with cc.AggregationQueue(max_batch=1000, max_delay_us=200_000) as q:
        futs = []

        def producer(t):
            for i in range(50):
                futs.append(q.submit_verify(bytes(32), bytes(32), bytes(64)))

        th = [threading.Thread(target=producer, args=(t,)) for t in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        futs.append(q.submit_batch(bytes(32), [(cc.PublicKey(), cc.Signature())] * 3))
        futs.append(q.submit_certificate(b"hdr", bytes(32), bytes(32), bytes(64), 1,
                                         [(cc.PublicKey(), cc.Signature())] * 2))
        futs.append(q.submit_digest(b"batch"))
        q.flush()
        assert all(f.done() for f in futs)
        for f in futs:
            with pytest.raises(cc.EngineError):
                f.result()
        st = q.stats()
        assert st["signatures"] == 200 and st["batches"] == 2 and st["digests"] == 1
        assert st["launches"] < 20  # coalesced, not one launch per request


@pytest.mark.gpu
def test_queue_verdicts_gpu(engine):
    vecs = [v for v in load_golden("verify_vectors.json") if len(v["msg"]) == 64]
    groups = load_golden("batch_vectors.json")
    with engine.AggregationQueue(max_batch=4096, max_delay_us=2000) as q:
        futs = []
        lock = threading.Lock()

        def producer(part):
            for v in part:
                f = q.submit_verify(bytes.fromhex(v["msg"]), bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]))
                with lock:
                    futs.append((f, v["expect"]))

        th = [threading.Thread(target=producer, args=(vecs[i::4],)) for i in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        gf = []
        for g in groups:
            if not g["expect"] and g["name"].startswith("small_order"):
                continue
            votes = [(engine.PublicKey(bytes.fromhex(p)), engine.Signature.from_bytes(bytes.fromhex(s)))
                     for p, s in zip(g["pks"], g["sigs"])]
            gf.append((q.submit_batch(bytes.fromhex(g["msg"]), votes), g["expect"]))
        for f, exp in futs + gf:
            assert f.result(timeout=60) == exp
        assert q.stats()["launches"] < len(futs)


@pytest.mark.gpu
@pytest.mark.parametrize("inline", ["1", "0"])
def test_queue_small_signature_windows_gpu(engine, monkeypatch, inline):
    """Windows of at most 16 signatures and nothing else take the latency
    kernel with the records in its arguments and the verdict words polled
    from page-locked memory (coa_queue_hip.cpp, coa_lat_verify_inline);
    COA_QUEUE_INLINE=0 stages them like larger windows.  Every golden vector
    (canonical, non-canonical, small-order, mixed-order...) in windows of
    1..16, both ways, gives the oracle's verdict."""
    monkeypatch.setenv("COA_QUEUE_INLINE", inline)
    vecs = [v for v in load_golden("verify_vectors.json") if len(v["msg"]) == 64]
    with engine.AggregationQueue(max_batch=4096, max_delay_us=2_000_000) as q:
        i, size = 0, 1
        while i < len(vecs):
            part = vecs[i:i + size]
            futs = [(q.submit_verify(bytes.fromhex(v["msg"]), bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"])),
                     v["expect"]) for v in part]
            q.flush()
            for f, exp in futs:
                assert f.result(timeout=30) == exp
            i += size
            size = size % 16 + 1
        m = q.metrics()
    assert m["windows"] >= 2 and m["failed_windows"] == 0


@pytest.mark.gpu
def test_queue_certificates_and_digests_gpu(engine):
    """Whole certificates (fused Certificate::verify crypto) and worker batch
    digests through the queue: one coalesced launch each, results equal the
    per-call entry points and hashlib."""
    import hashlib

    import certificates as C
    import workloads

    committee, batch = C.synth_certificates(12, committee_size=10, n_payload=4, seed=21)
    committee.register()
    batch.vote_sigs[3 * 7 + 2, 40] ^= 1          # certificate 3: bad vote
    batch.header_sigs[5, 33] ^= 1                 # certificate 5: bad header signature
    want = C.verify_certificate_batch(batch, committee, rng_seed=1)
    with engine.AggregationQueue(max_batch=100_000, max_delay_us=200_000) as q:
        cf = []
        for i in range(len(batch)):
            lo, hi = int(batch.offsets[i]), int(batch.offsets[i + 1])
            votes = [(engine.PublicKey(bytes(batch.vote_pks[j])), engine.Signature.from_bytes(bytes(batch.vote_sigs[j])))
                     for j in range(lo, hi)]
            cf.append(q.submit_certificate(batch.header_inputs[i], bytes(batch.ids[i]), bytes(batch.authors[i]),
                                           bytes(batch.header_sigs[i]), batch.round, votes))
        blobs = [workloads.worker_batch(b, ntx=20) for b in range(6)] + [b"", b"x" * 111, b"y" * 112]
        df = [q.submit_digest(b) for b in blobs]
        q.flush()
        got = [f.result(timeout=60) for f in cf]
        assert [int(g != 0) for g in got] == list(want)
        assert got[3] == engine.CERT_BAD_VOTES and got[5] == engine.CERT_BAD_HEADER_SIG
        assert [bytes(f.result(timeout=60)) for f in df] == [hashlib.sha512(b).digest()[:32] for b in blobs]
        st = q.stats()
        assert st["batches"] == len(batch) and st["digests"] == len(blobs) and st["launches"] <= 2


@pytest.mark.gpu
@pytest.mark.parametrize("inline", ["1", "0"])
def test_queue_small_certificate_windows_gpu(engine, monkeypatch, inline):
    """Windows of a few certificates and nothing else take the latency kernel
    with its last block writing the status words into page-locked memory,
    the arrays in the kernel arguments when they fit (C1's committee of 4:
    ~0.6 KB a certificate), else one copy (coa_queue_hip.cpp Slot::cpub,
    coa_certificate_verify_publish); COA_QUEUE_INLINE=0 stages them.  Windows
    of 1, 2 and 3 certificates with a bad vote (left open by the fused
    kernel, decided by the resolver), a bad header signature and a bad header
    id give the same bits as the host path, both ways."""
    import certificates as C

    monkeypatch.setenv("COA_QUEUE_INLINE", inline)
    committee, batch = C.synth_certificates(9, committee_size=4, n_payload=1, seed=29)
    committee.register()
    batch.vote_sigs[int(batch.offsets[1]) + 1, 40] ^= 1   # certificate 1: bad vote
    batch.header_sigs[4, 33] ^= 1                          # certificate 4: bad header signature
    h = bytearray(batch.header_inputs[6]); h[-1] ^= 1; batch.header_inputs[6] = bytes(h)  # 6: bad id
    want = C.verify_certificate_batch(batch, committee, rng_seed=1)
    with engine.AggregationQueue(max_batch=4096, max_delay_us=2_000_000) as q:
        got, i, size = [], 0, 1
        while i < len(batch):
            fs = []
            for c in range(i, min(i + size, len(batch))):
                lo, hi = int(batch.offsets[c]), int(batch.offsets[c + 1])
                votes = [(engine.PublicKey(bytes(batch.vote_pks[j])),
                          engine.Signature.from_bytes(bytes(batch.vote_sigs[j]))) for j in range(lo, hi)]
                fs.append(q.submit_certificate(batch.header_inputs[c], bytes(batch.ids[c]), bytes(batch.authors[c]),
                                               bytes(batch.header_sigs[c]), batch.round, votes))
            q.flush()
            got += [f.result(timeout=60) for f in fs]
            i += size
            size = size % 3 + 1
        m = q.metrics()
    assert [int(g != 0) for g in got] == list(want)
    assert got[1] == engine.CERT_BAD_VOTES and got[4] == engine.CERT_BAD_HEADER_SIG and got[6] & engine.CERT_BAD_HEADER_ID
    assert m["failed_windows"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("borrow", [False, True])
def test_queue_pipelined_windows_gpu(engine, borrow):
    """Many small windows in a row (max_batch 256) from four producers mixing
    every kind: windows overlap on the device slots (max_in_flight 2..8),
    every answer equals its expectation -- valid/corrupted signatures,
    certificates including ones that need the exact host re-decision (a vote
    key outside the registered committee, a corrupted vote), digests -- and
    the metrics account for every request."""
    import hashlib
    import struct

    import certificates as C
    import workloads

    n = 3000
    seeds, msgs = workloads.key_seeds(n, 40_000), workloads.messages(n, 40_000)
    pks, sigs = engine.sign_many(seeds, msgs)
    bad = np.zeros(n, bool)
    bad[::10] = True
    sigs[bad, 40] ^= 1
    committee, batch = C.synth_certificates(24, committee_size=10, n_payload=2, seed=5)
    committee.register()
    # certificate 4: one vote by a key outside the committee, validly signed (uncached -> host path, Ok)
    lo = int(batch.offsets[4])
    p_out, s_out = engine.sign_many(workloads.key_seeds(1, 99_999), batch.cert_digests[4:5])
    batch.vote_pks[lo], batch.vote_sigs[lo] = p_out[0], s_out[0]
    batch.vote_sigs[int(batch.offsets[9]) + 1, 50] ^= 1  # certificate 9: bad vote
    want_cert = [0] * len(batch)
    want_cert[9] = engine.CERT_BAD_VOTES
    blobs = [struct.pack("<Q", i) * (1 + i % 50) for i in range(300)]
    results = []
    lock = threading.Lock()
    with engine.AggregationQueue(max_batch=256, max_delay_us=300) as q:
        def producer(t):
            out = []
            for i in range(t, n, 4):
                sg = engine.Signature.from_bytes(bytes(sigs[i]))
                out.append(("sig", q.submit_verify(bytes(msgs[i]), bytes(pks[i]), sg), not bad[i]))
                if i % 100 == t and i // 100 < len(batch):
                    c = i // 100
                    lo_, hi_ = int(batch.offsets[c]), int(batch.offsets[c + 1])
                    votes = [(engine.PublicKey(bytes(batch.vote_pks[j])),
                              engine.Signature.from_bytes(bytes(batch.vote_sigs[j]))) for j in range(lo_, hi_)]
                    out.append(("cert", q.submit_certificate(batch.header_inputs[c], bytes(batch.ids[c]),
                                                             bytes(batch.authors[c]), bytes(batch.header_sigs[c]),
                                                             batch.round, votes, borrow=borrow), want_cert[c]))
                if i % 10 == t and i // 10 < len(blobs):
                    b = blobs[i // 10]
                    out.append(("dig", q.submit_digest(b), hashlib.sha512(b).digest()[:32]))
            with lock:
                results.extend(out)

        th = [threading.Thread(target=producer, args=(t,)) for t in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        q.flush()
        for kind, f, exp in results:
            got = f.result(timeout=120)
            if kind == "dig":
                assert bytes(got) == exp
            else:
                assert got == exp, (kind, got, exp)
        m = q.metrics()
        q.metrics_reset()
        m0 = q.metrics()
    assert m["requests"] == len(results) and m["signatures"] == n
    # pipelined over the slots (per GPU: 4 for verdicts, 8 for digests)
    assert m["windows"] > 4 and 2 <= m["max_in_flight"] <= 8
    assert 0 < m["wait_us_p50"] <= m["wait_us_p99"] <= m["wait_us_max"] * 1.1
    # per-stage time (COA_QSTAGE_*): every stage a window passes through was
    # timed; certificate 4's foreign key went through the resolver
    st = m["stage_us"]
    assert all(st[k] > 0 for k in ("intake", "gather", "pack", "enqueue", "device_wait", "callbacks", "resolve"))
    assert m["deferred_requests"] >= 1 and m["resolver_passes"] >= 1
    assert m0["requests"] == 0 and m0["windows"] == 0 and sum(m0["stage_us"].values()) == 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["api", "env"])
def test_queue_idle_launch_gpu(engine, monkeypatch, mode):
    """Idle launch (coa_queue_set_idle_launch(q, 1), or COA_QUEUE_IDLE_LAUNCH=1
    at creation): a request arriving while no window is in flight launches at
    once instead of waiting out max_delay_us (2 s here); one request at a
    time, each awaited before the next, answers exactly."""
    import time

    if mode == "env":
        monkeypatch.setenv("COA_QUEUE_IDLE_LAUNCH", "1")
    vecs = [v for v in load_golden("verify_vectors.json") if len(v["msg"]) == 64][:24]
    with engine.AggregationQueue(max_batch=4096, max_delay_us=2_000_000) as q:
        if mode == "api":
            q.set_idle_launch(1)
        t0 = time.perf_counter()
        for v in vecs:
            f = q.submit_verify(bytes.fromhex(v["msg"]), bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]))
            assert f.result(timeout=30) == v["expect"]
        el = time.perf_counter() - t0
        m = q.metrics()
    assert el < 2.0, el  # the deadline policy would take 24 x 2 s
    assert m["windows"] == len(vecs)


@pytest.mark.gpu
def test_queue_submit_from_callback_gpu(engine):
    """A verdict callback that submits the next request (the Rust service's
    continuations do): the callback runs on the queue's completion thread,
    which never launches a window itself (coa_queue.cpp t_queue_thread), so
    the collector launches it once the finishing window leaves the slot.
    24 chained requests under idle launch, each submitted from the previous
    one's callback, answer exactly and without waiting out the 2 s
    deadline."""
    import time

    vecs = [v for v in load_golden("verify_vectors.json") if len(v["msg"]) == 64][:24]
    got, done = [], threading.Event()
    with engine.AggregationQueue(max_batch=4096, max_delay_us=2_000_000) as q:
        q.set_idle_launch(1)

        def submit(i):
            v = vecs[i]
            f = q.submit_verify(bytes.fromhex(v["msg"]), bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]))
            f.add_done_callback(lambda f, i=i: on_done(i, f))

        def on_done(i, f):
            got.append((i, f.exception() or f.result()))
            if i + 1 < len(vecs):
                submit(i + 1)
            else:
                done.set()

        t0 = time.perf_counter()
        submit(0)
        assert done.wait(30)
        el = time.perf_counter() - t0
        m = q.metrics()
    assert [i for i, _ in got] == list(range(len(vecs)))
    assert [r for _, r in got] == [v["expect"] for v in vecs]
    assert el < 2.0, el  # one deadline wait would be 2 s
    assert m["windows"] == len(vecs) and m["failed_windows"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("borrow", [False, True])
def test_open_certificate_does_not_hold_its_window_gpu(engine, borrow):
    """A window holding one certificate with a vote key outside the registered
    committee (validly signed: the fused kernel cannot decide it, the exact
    path says Ok) answers every other request first: the open certificate
    goes to the lane's resolver (coa_certificate_resolve_raw), and every
    verdict still equals the C oracle's (oracle/coa_oracle.c, dalek's checks
    run per certificate -- primary/src/messages.rs:189-215)."""
    import os

    import certificates as C
    import coa_oracle as co
    import workloads

    committee, b = C.synth_certificates(16, committee_size=10, n_payload=2, seed=9)
    committee.register()
    lo = int(b.offsets[6])
    p_out, s_out = engine.sign_many(workloads.key_seeds(1, 77_777), b.cert_digests[6:7])
    b.vote_pks[lo], b.vote_sigs[lo] = p_out[0], s_out[0]   # certificate 6: open, Ok
    b.vote_sigs[int(b.offsets[11]) + 2, 45] ^= 1             # certificate 11: bad vote (open, then Err)
    zs = np.random.default_rng(3).integers(0, 256, (int(b.offsets[-1]), 16), dtype=np.uint8)
    exp = co.certificate_verify_many(list(b.header_inputs), b.ids, b.authors, b.header_sigs, b.round, b.vote_pks,
                                     b.vote_sigs, b.offsets, zs, min(8, os.cpu_count() or 1))
    n = 64
    seeds, msgs = workloads.key_seeds(n, 50_000), workloads.messages(n, 50_000)
    pks, sigs = engine.sign_many(seeds, msgs)
    sigs[::9, 40] ^= 1
    order, lock = [], threading.Lock()

    def done(tag):
        def cb(_f):
            with lock:
                order.append(tag)
        return cb

    with engine.AggregationQueue(max_batch=1 << 20, max_delay_us=2_000_000) as q:
        futs = []
        for i in range(len(b)):
            votes = [(engine.PublicKey(bytes(b.vote_pks[j])), engine.Signature.from_bytes(bytes(b.vote_sigs[j])))
                     for j in range(int(b.offsets[i]), int(b.offsets[i + 1]))]
            f = q.submit_certificate(b.header_inputs[i], bytes(b.ids[i]), bytes(b.authors[i]),
                                     bytes(b.header_sigs[i]), b.round, votes, borrow=borrow)
            f.add_done_callback(done(("cert", i)))
            futs.append((f, int(exp[i])))
        for i in range(n):
            f = q.submit_verify(bytes(msgs[i]), bytes(pks[i]), engine.Signature.from_bytes(bytes(sigs[i])))
            f.add_done_callback(done(("sig", i)))
            futs.append((f, i % 9 != 0))
        q.flush()
        for f, want in futs:
            assert f.result(timeout=60) == want
        m = q.metrics()
    assert exp[6] == 0 and exp[11] == engine.CERT_BAD_VOTES
    # two open certificates: 6 (a key outside the committee) and 11 (its
    # corrupted vote fails its own equation: inconclusive until the exact
    # random-linear-combination check, which may not assume R torsion-free)
    assert m["windows"] == 1 and m["deferred_requests"] == 2 and m["resolver_passes"] == 1
    # they are the last answers of their window, decided in one resolver pass
    assert set(order[-2:]) == {("cert", 6), ("cert", 11)}, order[-5:]
    assert len(order) == len(futs)


@pytest.mark.gpu
def test_cold_lane_set_up_by_its_first_window_gpu(engine, monkeypatch):
    """COA_QUEUE_LANES=verify (a primary never hashes worker
    batches): only the verify lane's slots are set up at creation; the digest
    lane's first window sets its own up, and its digests are still exact."""
    import hashlib

    monkeypatch.setenv("COA_QUEUE_LANES", "verify")
    vecs = [v for v in load_golden("verify_vectors.json") if len(v["msg"]) == 64][:8]
    with engine.AggregationQueue(max_batch=4096, max_delay_us=200) as q:
        fs = [(q.submit_verify(bytes.fromhex(v["msg"]), bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"])), v["expect"])
              for v in vecs]
        blobs = [b"cold lane", b"x" * 1000]
        ds = [q.submit_digest(b) for b in blobs]
        q.flush()
        assert [f.result(timeout=60) for f, _ in fs] == [e for _, e in fs]
        assert [bytes(d.result(timeout=60)) for d in ds] == [hashlib.sha512(b).digest()[:32] for b in blobs]
