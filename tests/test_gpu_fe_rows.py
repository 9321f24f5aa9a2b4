"""Row-parallel field arithmetic (csrc/coa_fe_wave.h: one GF(2^255-19)
element over a 16-lane DPP row) against the one-lane arithmetic of
coa_fe.h, on the device: z^((p-5)/8), z^(p-2), products, sums, differences and whole
decompressions (curve25519-dalek's sqrt_ratio_i chain), over random values,
carry-heavy limb patterns and the encodings the adversarial suite uses."""
import numpy as np
import pytest

import ed25519_ref as o

pytestmark = pytest.mark.gpu

P = 2**255 - 19


def _edge_values():
    vals = [0, 1, 2, P - 1, P, P + 1, 2**255 - 1, 2**256 - 1, 2**255, 2**32 - 1, 2**224 * (2**32 - 1),
            sum(0xFFFFFFFF << (32 * i) for i in range(0, 8, 2)), 38, 19, (P - 1) // 2]
    vals += [int.from_bytes(bytes([0xFF] * k + [0] * (32 - k)), "little") for k in range(1, 33)]
    vals += [int.from_bytes(T, "little") for T in (o.compress(t) for t in o.torsion_points())]
    vals.append(int.from_bytes(o.compress(o.B), "little"))
    return vals


def test_rows_match_one_lane(engine):
    import torch

    rng = np.random.default_rng(7)
    vals = [v.to_bytes(32, "little") for v in _edge_values()]
    rand = rng.integers(0, 256, (4096, 32), dtype=np.uint8)
    arr = np.concatenate([np.frombuffer(b"".join(vals), np.uint8).reshape(-1, 32), rand])
    # valid encodings too (decompression success path): public keys
    from workloads import key_seeds

    pks = np.stack([np.frombuffer(o.public_key(bytes(s)), np.uint8) for s in key_seeds(64)])
    arr = np.concatenate([arr, pks])
    dev = torch.device("cuda", 0)
    d_in = torch.from_numpy(arr.copy()).to(dev)
    out = torch.full((arr.shape[0],), -1, dtype=torch.int32, device=dev)
    engine.fe_rows_check_device(0, d_in, out)
    torch.cuda.synchronize()
    o_h = out.cpu().numpy()
    bad = np.nonzero(o_h)[0]
    assert bad.size == 0, [(int(i), int(o_h[i]), arr[i].tobytes().hex()) for i in bad[:8]]
