"""CPU: a C program compiled with gcc against include/coa_verify.h
(-std=c11 -Wall -Wextra -Werror) calls every entry point of the engine's C
ABI, so the header's prototypes -- not only the exported symbol names -- are
checked; run without a GPU it checks that every device call refuses with
COA_ENODEVICE (no CPU fallback) and that the host-only calls behave.  The GPU
form of the same harness runs in tests/test_gpu_c_abi.py.

The multi-producer queue harness (tests/c_abi/queue_harness.c, the way the
Rust VerifyService drives the queue) is compiled the same way; without a GPU
every one of its requests must still be answered, with the engine error."""
import json
import os
import struct
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


QSRC = os.path.join(ROOT, "tests", "c_abi", "queue_harness.c")
QOUT = os.path.join(ROOT, "tests", "c_abi", "queue_harness")


def build_queue_harness():
    import build

    lib = build.build()
    libdir = os.path.dirname(lib)
    tmp = f"{QOUT}.{os.getpid()}"
    cmd = ["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-O2", "-pthread", "-I", os.path.join(ROOT, "include"),
           QSRC, "-o", tmp, "-L", libdir, "-lcoa_verify", f"-Wl,-rpath,{libdir}", "-L/opt/rocm/lib",
           "-Wl,-rpath,/opt/rocm/lib"]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    os.replace(tmp, QOUT)
    return QOUT


def write_queue_vectors(path):
    """The golden verify vectors with 32-byte messages (crypto API), the
    golden batch groups (z-independent verdicts) and SHA-512 vectors, in the
    queue harness's binary format; returns (n_verify, n_batch, n_digest)."""
    gold = os.path.join(ROOT, "tests", "golden")
    vv = [v for v in json.load(open(os.path.join(gold, "verify_vectors.json"))) if len(v["msg"]) == 64]
    bv = json.load(open(os.path.join(gold, "batch_vectors.json")))
    dv = json.load(open(os.path.join(gold, "sha512_vectors.json")))
    out = [struct.pack("<4I", 0x51414F43, len(vv), len(bv), len(dv))]
    for v in vv:
        out.append(bytes.fromhex(v["msg"]) + bytes.fromhex(v["pk"]) + bytes.fromhex(v["sig"]) +
                   bytes([0 if v["expect"] else 1]))
    for g in bv:
        out.append(bytes.fromhex(g["msg"]) + struct.pack("<I", len(g["pks"])) + bytes([0 if g["expect"] else 1]))
        for pk, sg in zip(g["pks"], g["sigs"]):
            out.append(bytes.fromhex(pk) + bytes.fromhex(sg))
    for d in dv:
        data = bytes.fromhex(d["msg"])
        out.append(struct.pack("<I", len(data)) + data + bytes.fromhex(d["sha512"])[:32])
    with open(path, "wb") as f:
        f.write(b"".join(out))
    return len(vv), len(bv), len(dv)


def test_queue_harness_cpu_mode(tmp_path):
    """No GPU: every request of 4 producers is answered exactly once, each
    with the engine error (the harness then exits 1)."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present: tests/test_gpu_queue_harness.py runs it")
    exe = build_queue_harness()
    vec = str(tmp_path / "vectors.bin")
    nv, nb, nd = write_queue_vectors(vec)
    r = subprocess.run([exe, vec, "4", "1"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 1, r.stderr
    res = json.loads(r.stdout.strip().splitlines()[-1])
    n = 4 * (nv + nb + nd)
    assert res["submitted"] == n and res["answered"] == n and res["bad_status"] == n, res
    assert res["retried_windows"] == 0  # "no device" is not a recoverable failure


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


WSRC = os.path.join(ROOT, "tests", "c_abi", "wire_queue_harness.c")
WOUT = os.path.join(ROOT, "tests", "c_abi", "wire_queue_harness")
WIRE_CERTS = os.path.join(ROOT, "tests", "golden", "wire_certificates.bin")


def build_wire_queue_harness():
    import build

    lib = build.build()
    libdir = os.path.dirname(lib)
    tmp = f"{WOUT}.{os.getpid()}"
    cmd = ["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-O2", "-pthread", "-I", os.path.join(ROOT, "include"),
           WSRC, "-o", tmp, "-L", libdir, "-lcoa_verify", f"-Wl,-rpath,{libdir}", "-L/opt/rocm/lib",
           "-Wl,-rpath,/opt/rocm/lib"]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    os.replace(tmp, WOUT)
    return WOUT


def test_wire_certificates_fixture_matches_oracle():
    """The committed frames decode (test encoder layout) and their expected
    bits are the C oracle's: regenerating gives the same file."""
    import hashlib

    with open(WIRE_CERTS, "rb") as f:
        blob = f.read()
    assert blob[:4] == b"CQWC"
    n_keys = struct.unpack_from("<I", blob, 4)[0]
    n = struct.unpack_from("<I", blob, 8 + 32 * n_keys)[0]
    assert n_keys == 4 and n == 20
    # the generator is deterministic: a fresh run reproduces the fixture
    import runpy
    import shutil
    import tempfile

    with tempfile.TemporaryDirectory() as td:
        gen = os.path.join(td, "gen.py")
        shutil.copy(os.path.join(ROOT, "tests", "golden", "make_wire_certificates.py"), gen)
        src = open(gen).read().replace('HERE = os.path.dirname(os.path.abspath(__file__))',
                                       f'HERE = {os.path.join(ROOT, "tests", "golden")!r}')
        src = src.replace('os.path.join(HERE, "wire_certificates.bin")', repr(os.path.join(td, "out.bin")))
        open(gen, "w").write(src)
        runpy.run_path(gen, run_name="__main__")
        assert hashlib.sha256(open(os.path.join(td, "out.bin"), "rb").read()).digest() == \
            hashlib.sha256(blob).digest()


def test_wire_queue_harness_cpu_mode():
    """No GPU: the native decoder still decodes every frame (host-only), and
    every queued certificate is answered once with the engine error."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present: tests/test_gpu_queue_harness.py runs it")
    exe = build_wire_queue_harness()
    r = subprocess.run([exe, WIRE_CERTS, "0", "2"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 1, r.stderr
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["decoded"] and res["frames"] == 20
    assert res["answered"] == res["submitted"] == 40 and res["bad_status"] == 40, res
