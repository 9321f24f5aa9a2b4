"""CPU: the Lehmer blocks of the scalar halving (xrpl-coa-prototype_amd/csrc/
coa_lehmer.h, used by coa_halve.h on the device) compiled for the host and
checked against an exact big-integer Euclidean algorithm on (8l, k): every
state a Lehmer block reaches must be a consecutive remainder pair of the
exact sequence, with the exact cofactor magnitudes, so the halving's
candidates -- and hence (c, d) -- are the ones the full-width steps find.
Random k, the adversarial k of tests/test_gpu_halve.py (quotients around
2^31, k near 8l/q, a large quotient late in the sequence) and tiny /
near-l k."""
import ctypes
import os
import random
import subprocess

import pytest

from conftest import ROOT

import ed25519_ref as o

L = o.L
SRC = os.path.join(ROOT, "tests", "lehmer", "lehmer_host.cpp")
INC = os.path.join(ROOT, "xrpl-coa-prototype_amd", "csrc")


@pytest.fixture(scope="module")
def lehmer(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("lehmer") / "liblehmer.so")
    subprocess.run(["g++", "-O2", "-shared", "-fPIC", "-I", INC, SRC, "-o", so], check=True)
    lib = ctypes.CDLL(so)
    P = ctypes.POINTER(ctypes.c_uint32)
    lib.lehmer_step.argtypes = [P, P, P, P, ctypes.c_int]
    lib.lehmer_step.restype = ctypes.c_int
    return lib


def _limbs(x):
    return (ctypes.c_uint32 * 8)(*[(x >> (32 * i)) & 0xFFFFFFFF for i in range(8)])


def _val(a):
    return sum(int(a[i]) << (32 * i) for i in range(8))


def _exact_sequence(k):
    r = [8 * L, k]
    t = [0, 1]  # magnitudes
    while r[-1]:
        q = r[-2] // r[-1]
        r.append(r[-2] - q * r[-1])
        t.append(t[-2] + q * t[-1])
    return r, t


def _run(lib, k, stop=140, final=124):
    r, t = _exact_sequence(k)
    a, b, ta, tb = _limbs(8 * L), _limbs(k), _limbs(0), _limbs(1)
    j, blocks, steps = 0, 0, 0
    while _val(b).bit_length() > final:
        n = lib.lehmer_step(a, b, ta, tb, stop) if _val(b).bit_length() > stop else 0
        if n:
            blocks += 1
            steps += n
            j += n
        else:  # one exact step
            av, bv, tav, tbv = _val(a), _val(b), _val(ta), _val(tb)
            q = av // bv
            a, b, ta, tb = _limbs(bv), _limbs(av - q * bv), _limbs(tbv), _limbs(tav + q * tbv)
            j += 1
        assert (_val(a), _val(b)) == (r[j], r[j + 1]), (hex(k), j)
        assert (_val(ta), _val(tb)) == (t[j], t[j + 1]), (hex(k), j)
    return blocks, steps, j


def _adversarial(rng):
    ks = [0x8d4cd933cbb871883dfcacf26cb47af3fff64fcce0664ba4450ab8083db849b, 1, 2, 3, 7, 8, L - 1, L - 2, L // 2,
          (1 << 252) - 1, (1 << 128) + 1, (1 << 127) - 1]
    for q in (2 ** 10, 2 ** 20, 2 ** 30, 2 ** 31 - 1, 2 ** 31, 2 ** 31 + 1, 2 ** 32 - 1, 2 ** 32, 3153881985,
              2 ** 40, 2 ** 60, 2 ** 100):
        base = 8 * L // q
        for d in (0, 1, -1, 2, rng.getrandbits(16)):
            ks.append((base + d) % L)
    for m in (3, 17, 1000):
        for Q in (2 ** 31, 2 ** 33, 2 ** 45):
            ks.append((8 * L * Q // (m * Q + 1)) % L)
    return [k for k in ks if k]


def test_lehmer_blocks_follow_the_exact_euclidean_sequence(lehmer):
    rng = random.Random(11)
    ks = _adversarial(rng) + [rng.randrange(1, L) for _ in range(3000)]
    tot_blocks = tot_steps = tot_all = 0
    for k in ks:
        blocks, steps, j = _run(lehmer, k)
        tot_blocks += blocks
        tot_steps += steps
        tot_all += j
    # random k: ~80 Euclid steps to 124 bits, almost all inside ~6 blocks
    assert tot_steps > 0.8 * tot_all
    assert tot_blocks < tot_steps / 8
