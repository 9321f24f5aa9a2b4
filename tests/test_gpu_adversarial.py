"""GPU parity at scale (C5 shape, reduced size): 1% adversarial items over
the 8 classes of SURVEY 8(d) among device-signed valid triples; verdicts must
equal the C restatement of dalek (oracle/coa_oracle.c) bit for bit."""
import os

import numpy as np
import pytest

import coa_oracle as co
from conftest import load_golden

pytestmark = pytest.mark.gpu


def _pool():
    return [(bytes.fromhex(v["msg"]), bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]))
            for v in load_golden("mixed_order_pool.json")]


@pytest.mark.parametrize("n,frac,il", [(4096, 0.25, None), (65_536, 0.01, None), (262_144, 0.01, None),
                                        (262_144, 0.01, "1")])
def test_adversarial_mix_bit_exact(engine, n, frac, il, monkeypatch):
    """n = 65,536 is the C2 size (the one-wave main kernel by default); 2^18
    takes the three-wave one by default and the one-wave one forced."""
    if il is not None:
        monkeypatch.setenv("COA_MAIN_IL", il)
    from workloads import adversarial_mix, key_seeds, messages

    seeds, msgs = key_seeds(n), messages(n)
    pks, sigs = engine.sign_many(seeds, msgs)
    msgs, pks, sigs, cls = adversarial_mix(msgs, pks, sigs, frac=frac, seed=0xC0A5, mixed_pool=_pool())
    got = engine.verify_strict_many(msgs, pks, sigs)
    threads = min(16, os.cpu_count() or 1)
    exp = co.verify_strict_many(msgs, pks, sigs, threads)
    mism = np.nonzero(got != exp)[0]
    assert mism.size == 0, [(int(i), int(cls[i])) for i in mism[:20]]
    # class sanity: every mutated class present, untouched items all accepted
    assert set(np.unique(cls[cls >= 0])) == set(range(8))
    assert (got[cls == -1] == 0).all()
    assert (got[cls == 7] == 0).all()


def test_adversarial_device_path(engine):
    """Same mix through the HBM-resident entry point on an explicit stream."""
    import torch

    from workloads import adversarial_mix, key_seeds, messages

    n = 8192
    pks, sigs = engine.sign_many(key_seeds(n, 100), messages(n, 100))
    msgs, pks, sigs, cls = adversarial_mix(messages(n, 100), pks, sigs, frac=0.1, seed=9, mixed_pool=_pool())
    exp = co.verify_strict_many(msgs, pks, sigs, min(16, os.cpu_count() or 1))
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    t = [torch.from_numpy(a).to(dev) for a in (msgs, pks, sigs)]
    out = torch.ones(n, dtype=torch.uint8, device=dev)
    ws = torch.empty(engine.verify_workspace_bytes(n), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    engine.verify_strict_many_device(0, t[0], t[1], t[2], out, ws, s)
    s.synchronize()
    assert (out.cpu().numpy() == exp).all()


VERIFY_PATHS = {
    "split": {},                                            # default: k_pre_halve + k_verify_main
    "split/narrow": {"COA_WCOMB": "0"},                     # [e]B from the radix-256 comb
    "split/plain-main": {"COA_MAIN_IL": "0", "COA_MAIN_TWO": "0"},  # k_verify_main without interleaved products
    "split/one-wave-main": {"COA_MAIN_TWO": "0"},           # k_verify_main<1, true> (C2's kernel)
    "split/two-wave-main": {"COA_MAIN_TWO": "1"},           # k_verify_main2 (default up to a quarter wave per SIMD)
    "split/eb-in-main": {"COA_SPLIT_EB": "0"},              # [e]B in k_verify_main, not k_pre_halve
    "split/eb-in-main/narrow": {"COA_SPLIT_EB": "0", "COA_WCOMB": "0"},
    "single": {"COA_VERIFY_SPLIT": "0"},                    # k_halve + k_verify_halved
    "single/narrow": {"COA_VERIFY_SPLIT": "0", "COA_WCOMB": "0"},
    "full": {"COA_VERIFY_IMPL": "full"},                    # k_hram + k_verify_strict, no halving
}


@pytest.mark.parametrize("impl", list(VERIFY_PATHS))
def test_every_verify_path_agrees(engine, impl, monkeypatch):
    """Every verification path (read per call) matches the oracle on the same
    adversarial mix: the split launch pair (default), the single-kernel
    halved path, the full-length kernel, each comb of B."""
    from workloads import adversarial_mix, key_seeds, messages

    for k, v in VERIFY_PATHS[impl].items():
        monkeypatch.setenv(k, v)
    n = 20_000
    pks, sigs = engine.sign_many(key_seeds(n, 7), messages(n, 7))
    msgs, pks, sigs, cls = adversarial_mix(messages(n, 7), pks, sigs, frac=0.05, seed=77, mixed_pool=_pool())
    got = engine.verify_strict_many(msgs, pks, sigs)
    exp = co.verify_strict_many(msgs, pks, sigs, min(16, os.cpu_count() or 1))
    assert (got == exp).all(), np.nonzero(got != exp)[0][:10]


@pytest.mark.parametrize("n", [1, 3, 255, 257, 769])
def test_split_path_ragged_small_calls(engine, n, monkeypatch):
    """The split kernels on call sizes around their block edges (one to three
    blocks per role of k_pre_halve, partial last blocks): COA_LAT_MAX=0 keeps
    these small calls off the latency route.  Adversarial mix vs the oracle."""
    from workloads import adversarial_mix, messages

    monkeypatch.setenv("COA_LAT_MAX", "0")
    m0 = messages(n, 31)
    pks, sigs = engine.sign_many(np.frombuffer(bytes(range(256)) * ((32 * n) // 256 + 1), np.uint8)[: 32 * n]
                                 .reshape(n, 32), m0)
    msgs, pks, sigs, _ = adversarial_mix(m0, pks, sigs, frac=0.3, seed=n, mixed_pool=_pool())
    got = engine.verify_strict_many(msgs, pks, sigs)
    exp = co.verify_strict_many(msgs, pks, sigs, 1)
    assert (got == exp).all(), np.nonzero(got != exp)[0][:10]


def test_adversarial_mix_streamed_through_the_queue(engine):
    """The C2-size adversarial mix (65,536 triples, 1 % over the 8 classes)
    submitted one signature per request through the aggregation queue from a
    C caller at 2 M requests/s (tools/latc.c latc_paced, max_batch 16,384:
    windows on the latency and the throughput kernels, backlog windows when
    the slots are busy): every callback's verdict equals the oracle's."""
    import bench
    from workloads import adversarial_mix, key_seeds, messages

    n = 65_536
    pks, sigs = engine.sign_many(key_seeds(n, 300_000), messages(n, 300_000))
    msgs, pks, sigs, cls = adversarial_mix(messages(n, 300_000), pks, sigs, frac=0.01, seed=0xC0A6,
                                           mixed_pool=_pool())
    exp = co.verify_strict_many(msgs, pks, sigs, min(16, os.cpu_count() or 1))
    assert set(np.unique(cls[cls >= 0])) == set(range(8))
    arrive = np.arange(n, dtype=np.float64) / 2e6
    # paced_queue asserts that every answer equals its expectation
    lat, el, met = bench.paced_queue(arrive, np.zeros(n, np.int32), np.arange(n, dtype=np.uint32), vm=msgs, vp=pks,
                                     vs=sigs, vexp=exp, max_batch=16384, max_delay_us=200)
    assert met["signatures"] == n and met["failed_windows"] == 0, met
    assert met["windows"] > 4
