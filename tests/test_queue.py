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
        q.flush()
        assert all(f.done() for f in futs)
        for f in futs:
            with pytest.raises(cc.EngineError):
                f.result()
        st = q.stats()
        assert st["signatures"] == 200 and st["batches"] == 1
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
