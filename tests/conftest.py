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
