"""CPU: a C program compiled with gcc against include/coa_verify.h
(-std=c11 -Wall -Wextra -Werror) calls every entry point of the engine's C
ABI, so the header's prototypes -- not only the exported symbol names -- are
checked; run without a GPU it checks that every device call refuses with
COA_ENODEVICE (no CPU fallback) and that the host-only calls behave.  The GPU
form of the same harness runs in tests/test_gpu_c_abi.py."""
import os
import subprocess

import pytest

from conftest import ROOT

SRC = os.path.join(ROOT, "tests", "c_abi", "abi_harness.c")
OUT = os.path.join(ROOT, "tests", "c_abi", "abi_harness")


def build_harness():
    import build

    lib = build.build()
    libdir = os.path.dirname(lib)
    # built under a per-process name and renamed into place, so concurrent
    # test processes never write an executable another one is running
    tmp = f"{OUT}.{os.getpid()}"
    cmd = ["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-pedantic", "-O1", "-I", os.path.join(ROOT, "include"),
           SRC, "-o", tmp, "-L", libdir, "-lcoa_verify", f"-Wl,-rpath,{libdir}", "-L/opt/rocm/lib",
           "-Wl,-rpath,/opt/rocm/lib"]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    os.replace(tmp, OUT)
    return OUT


def test_harness_compiles_against_header():
    assert os.path.exists(build_harness())


def test_harness_cpu_mode():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present: tests/test_gpu_c_abi.py runs the gpu mode")
    exe = build_harness()
    r = subprocess.run([exe, "cpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "abi harness ok (cpu)" in r.stdout
