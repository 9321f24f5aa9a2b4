"""GPU: the multi-producer queue harness (tests/c_abi/queue_harness.c, built
on the CPU by tests/test_c_abi.py) -- several C producer threads submit the
golden verify vectors (single and in groups of 8), the golden vote batches
and SHA-512 vectors through coa_queue_submit_* with completion callbacks, as
the Rust VerifyService does (rust/crypto/src/service.rs); every callback
compares its verdict / digest with the golden expectation.  Then the same
with injected launch failures (COA_QUEUE_FAULT): every failed window is
re-run on the recovery context and still answered exactly."""
import json
import os
import subprocess

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _run(tmp_path, producers, rounds, env_extra=None, max_batch=4096, delay=500):
    from test_c_abi import QOUT, build_queue_harness, write_queue_vectors

    exe = QOUT if os.path.exists(QOUT) else build_queue_harness()
    vec = str(tmp_path / "vectors.bin")
    nv, nb, nd = write_queue_vectors(vec)
    env = dict(os.environ, **(env_extra or {}))
    r = subprocess.run([exe, vec, str(producers), str(rounds), str(max_batch), str(delay)], capture_output=True,
                       text=True, timeout=300, env=env)
    res = json.loads(r.stdout.strip().splitlines()[-1]) if r.stdout.strip() else {}
    assert r.returncode == 0, (res, r.stderr[-3000:])
    assert res["submitted"] == producers * rounds * (nv + nb + nd)
    return res


def test_queue_harness_many_producers_golden(tmp_path):
    res = _run(tmp_path, producers=8, rounds=4)
    assert res["wrong"] == 0 and res["bad_status"] == 0
    assert res["windows"] < res["submitted"] // 8  # coalesced
    assert res["retried_windows"] == 0 and res["failed_windows"] == 0


def test_queue_harness_recovers_injected_failures(tmp_path):
    """Every 3rd window's launch fails after its input copy is enqueued; the
    slot is rebuilt and the window re-run on the recovery context."""
    res = _run(tmp_path, producers=4, rounds=4, env_extra={"COA_QUEUE_FAULT": "3"}, max_batch=256, delay=200)
    assert res["wrong"] == 0 and res["bad_status"] == 0
    assert res["retried_windows"] >= 1 and res["recovered_windows"] == res["retried_windows"], res
    assert res["failed_windows"] == 0


@pytest.mark.parametrize("register", [1, 0])
def test_wire_frames_decoded_and_queued_golden(register):
    """Raw PrimaryMessage::Certificate frames (tests/golden/wire_certificates.bin)
    through the native decoder (coa_wire_scan / coa_wire_decode_certificates)
    into coa_queue_submit_certificate, from C: every status equals the
    oracle's bits, with the committee registered (fused cached kernel; the
    outside-key certificates re-decided exactly) and without (uncached path)."""
    from test_c_abi import WIRE_CERTS, WOUT, build_wire_queue_harness

    exe = WOUT if os.path.exists(WOUT) else build_wire_queue_harness()
    r = subprocess.run([exe, WIRE_CERTS, str(register), "3"], capture_output=True, text=True, timeout=300)
    res = json.loads(r.stdout.strip().splitlines()[-1]) if r.stdout.strip() else {}
    assert r.returncode == 0, (res, r.stderr[-3000:])
    assert res["decoded"] and res["answered"] == 60 and res["wrong"] == 0 and res["failed_windows"] == 0


def test_queue_harness_backlog_windows(tmp_path):
    """Backlog windows (coa_queue.cpp Lane::backlog_batch): one verdict slot,
    64-item windows, 8 C producers submitting faster than the slot drains
    them.  A window closed while the slot is busy waits for it and takes the
    backlog (up to 2,048 items here); every answer still equals the golden
    one, and some window outgrew what a shard-bounded window can hold (two
    shards of < max_batch items plus one request)."""
    gold = os.path.join(ROOT, "tests", "golden", "batch_vectors.json")
    largest = max(len(g["pks"]) for g in json.load(open(gold)))
    env = {"COA_QUEUE_SLOTS": "1", "COA_QUEUE_BACKLOG_BATCH": "2048", "COA_QUEUE_BACKLOG_MIN": "1"}
    res = _run(tmp_path, producers=8, rounds=16, env_extra=env, max_batch=64, delay=200)
    assert res["wrong"] == 0 and res["bad_status"] == 0, res
    assert res["failed_windows"] == 0
    assert res["max_window"] > 2 * 64 + max(8, largest), res
