"""GPU: the halved-scalar verify path on challenge scalars k that stress the
half-gcd of k_halve (csrc/coa_halved.hip): Euclid quotients around and above
2^31 (the f64-estimate / shift-subtract boundary), k near multiples of 8l/q,
tiny and near-l scalars.  Valid (k, A, R, s) are built for ARBITRARY k
(s = r + k a mod l, A = aB, R = rB) and go through
coa_ed25519_verify_prehashed_many_device, so the kernel sees exactly these k;
every valid tuple must be accepted and every s+1 variant rejected.

Regression: one valid signature in 4M of the C5 set was rejected when the
quotient estimate used v_rcp_f64 (its k has a 32-bit quotient); that k is
pinned below."""
import random

import numpy as np
import pytest

import ed25519_ref as o

pytestmark = pytest.mark.gpu

L = o.L
C5_K = 0x8d4cd933cbb871883dfcacf26cb47af3fff64fcce0664ba4450ab8083db849b  # C5 index 1508773 (4M run)


def _ks(rng):
    ks = [C5_K, 1, 2, 3, 7, 8, L - 1, L - 2, L // 2, (1 << 252) - 1, (1 << 128) + 1, (1 << 127) - 1]
    for q in (2 ** 10, 2 ** 20, 2 ** 30, 2 ** 31 - 1, 2 ** 31, 2 ** 31 + 1, 2 ** 32 - 1, 2 ** 32, 3153881985,
              2 ** 40, 2 ** 60, 2 ** 100):
        base = 8 * L // q
        for d in (0, 1, -1, 2, rng.getrandbits(16)):
            ks.append((base + d) % L)
    # a large quotient at a LATER Euclid step: k = 8l / (m + 1/Q) style
    for m in (3, 17, 1000):
        for Q in (2 ** 31, 2 ** 33, 2 ** 45):
            ks.append((8 * L * Q // (m * Q + 1)) % L)
    ks += [rng.randrange(1, L) for _ in range(24)]
    return [k for k in ks if k]


def test_halved_path_on_adversarial_k(engine):
    import torch

    rng = random.Random(7)
    ks = _ks(rng)
    kb, pks, sigs, expect = [], [], [], []
    for i, k in enumerate(ks):
        a = rng.randrange(1, L)
        r = rng.randrange(1, L)
        A = o.compress(o.pmul(a, o.B))
        R = o.compress(o.pmul(r, o.B))
        s = (r + k * a) % L
        for bad in (False, True):
            ss = (s + 1) % L if bad else s
            kb.append(k.to_bytes(32, "little"))
            pks.append(A)
            sigs.append(R + ss.to_bytes(32, "little"))
            expect.append(1 if bad else 0)
    n = len(kb)
    dev = torch.device("cuda", 0)
    T = lambda bs, w: torch.from_numpy(np.frombuffer(b"".join(bs), np.uint8).reshape(n, w).copy()).to(dev)  # noqa
    out = torch.full((n,), 7, dtype=torch.uint8, device=dev)
    stream = torch.cuda.Stream(dev)
    engine.verify_prehashed_many_device(0, T(kb, 32), T(pks, 32), T(sigs, 64), out, None, stream)
    stream.synchronize()
    got = out.cpu().numpy().tolist()
    bad = [(hex(int.from_bytes(kb[i], "little")), got[i], expect[i]) for i in range(n) if got[i] != expect[i]]
    assert not bad, bad[:8]
