"""CPU: the C-ABI library builds for gfx950, loads, exports every symbol that
include/coa_verify.h declares, and -- with no GPU present -- refuses work with
COA_ENODEVICE instead of computing anything on the CPU."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "coa_verify.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(coa_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def libpath():
    import build

    return build.build()


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("coa_ed25519_verify_strict", "coa_ed25519_verify_strict_many", "coa_ed25519_verify_batch",
              "coa_ed25519_verify_batch_groups", "coa_sha512_many", "coa_sha512_trunc32_many"):
        assert s in syms


def test_library_exports_every_declared_symbol(libpath):
    lib = ctypes.CDLL(libpath)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_python_mirror_binds_every_symbol(libpath):
    import coa_crypto

    L = coa_crypto.lib()
    for s in declared_symbols():
        assert getattr(L, s).restype is not None or s == "coa_shutdown"


def test_no_cpu_fallback_without_gpu(libpath):
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu tests")
    lib = ctypes.CDLL(libpath)
    lib.coa_init.restype = ctypes.c_int
    assert lib.coa_init(0) == -2  # COA_ENODEVICE
    buf = (ctypes.c_uint8 * 128)()
    lib.coa_ed25519_verify_strict.restype = ctypes.c_int
    assert lib.coa_ed25519_verify_strict(buf, buf, buf) == -2


def test_mirror_raises_loudly_without_gpu(libpath):
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import coa_crypto

    with pytest.raises(coa_crypto.EngineError):
        coa_crypto.Signature().verify(coa_crypto.Digest(), coa_crypto.PublicKey())
