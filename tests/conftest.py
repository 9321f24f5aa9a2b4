"""Shared test setup.

* registers the `gpu` marker (tests that need an MI355X; `-m "not gpu"` runs
  the rest on CPU),
* puts the engine's Python mirror (xrpl-coa-prototype_amd/coa_crypto) and the
  CPU oracle (oracle/, test infrastructure only) on sys.path,
* loads the committed golden fixtures (tests/golden/*.json).
"""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "xrpl-coa-prototype_amd")
for p in (PKG, os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def engine():
    """The built engine library, initialised on the GPU (gpu tests only).

    torch is imported first: the engine links libamdhip64 by soname, so the
    process then holds one HIP runtime (torch's).  Loaded the other way round,
    torch's bundled runtime is a second copy that sees no GPU
    (tools/probe_torch_after_init.py)."""
    import torch  # noqa: F401

    import build  # xrpl-coa-prototype_amd/build.py

    build.build()
    import coa_crypto

    coa_crypto.init(0)
    return coa_crypto


@pytest.fixture(autouse=True)
def _kfd_queue_trace(request):
    """COA_TRACE_KFD_QUEUES=1 (diagnostics only): print how many hardware
    queues the kernel driver holds for this process before and after each
    test (/sys/class/kfd/kfd/proc/<pid>/queues) -- a process whose queues
    outnumber what the GPU's scheduler maps at once is time-sliced."""
    if os.environ.get("COA_TRACE_KFD_QUEUES") != "1":
        yield
        return
    path = f"/sys/class/kfd/kfd/proc/{os.getpid()}/queues"

    def count():
        try:
            return len(os.listdir(path))
        except OSError as e:
            return f"n/a ({e.__class__.__name__})"

    before = count()
    yield
    print(f"\n[kfd queues] {request.node.name}: {before} -> {count()}", file=sys.stderr, flush=True)


@pytest.fixture(autouse=True, scope="session")
def _gc_pause_trace():
    """COA_TRACE_GC=1 (diagnostics only): print every Python garbage
    collection that held the interpreter for more than 5 ms, with its
    CLOCK_MONOTONIC time (the clock of the queue's COA_QUEUE_TRACE_SLOW_US
    lines): a queue callback into Python waits for the GIL that long."""
    if os.environ.get("COA_TRACE_GC") != "1":
        yield
        return
    import gc
    import time

    t0 = {}

    def cb(phase, info):
        if phase == "start":
            t0["t"] = time.monotonic()
        else:
            dt = time.monotonic() - t0.get("t", time.monotonic())
            if dt > 0.005:
                print(f"\n[gc] generation {info['generation']} pause {dt * 1e3:.1f} ms at t={t0['t']:.6f} s "
                      f"({info['collected']} collected)", file=sys.stderr, flush=True)

    gc.callbacks.append(cb)
    yield
    gc.callbacks.remove(cb)
