"""GPU: the C harness (tests/c_abi/abi_harness.c, built on the CPU by
tests/test_c_abi.py) in gpu mode -- every entry point called from C, the
reference's "Hello, world!" signature Ok and a corrupted copy Err through the
verify entry points, RFC 8032 signing reproduces it."""
import os
import subprocess

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_harness_gpu_mode():
    exe = os.path.join(ROOT, "tests", "c_abi", "abi_harness")
    if not os.path.exists(exe):
        from test_c_abi import build_harness

        exe = build_harness()
    r = subprocess.run([exe, "gpu"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "abi harness ok (gpu)" in r.stdout
