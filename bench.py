"""Benchmark: ed25519 verifications/sec on MI355X (BASELINE.json `metric`).

Workload (N=1, BASELINE.json configs[1], "C2"): 65,536 independent
(32 B digest, pk, sig) triples, all valid, one key per signature, per-signature
verify (crypto::Signature::verify == dalek verify_strict).  Inputs are
synthesised with the reference's byte formats (workloads.py), signed on the
device, and are resident in HBM before the timed region.

A step = one pass of the hot path over the batch: one
coa_ed25519_verify_strict_many_device call (k = SHA-512(R||A||M) mod l, the
halving, decompressions and tables in k_pre_halve, the joint pass in
k_verify_main).  With N GPUs every rank
verifies its own 65,536 triples (weak scaling, contiguous index ranges, no
data-path collective); value = all ranks' verifications / max-over-ranks time.

Also reported:
  roofline      the verify call (k_pre_halve + k_verify_main) against the
                INT32 VALU issue peak; algorithmic work = the dalek
                algorithm's field operation count (2,967 mul+sq per verify,
                frozen by the instrumented C restatement: oracle/coa_oracle.c)
                x 200 INT32 ops per field op (SURVEY.md 8(d) cost model); its
                time is measured here with HIP events on the stream it runs on.
  cpu_baseline  the C restatement of dalek's algorithms (oracle/, "port")
                on this host's cores, rank 0 at N=1 only, on a bounded sample.
  secondary     (rank 0, N=1) one C5 shard (2^21 triples) per verify call;
                verify_batch through the Pippenger kernels (one 2^21-signature
                group; one certificate's 67 votes, p50 beside the CPU);
                C4 worker-batch SHA-512 GB/s; C3 and C1
                Certificate::verify -- certificates/s for a round resident in
                HBM and p50/p99 latency of one certificate through the
                host-pointer C ABI, beside the single-core CPU restatement.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "xrpl-coa-prototype_amd")
sys.path.insert(0, PKG)

# dalek algorithm field operations per verify_strict (fe_mul + fe_sq), measured
# by oracle/_build/libcoa_oracle_count.so over the golden valid vectors.
FIELD_OPS_PER_VERIFY = 2967
INT32_OPS_PER_FIELD_OP = 200
ALG_INT32_OPS_PER_VERIFY = FIELD_OPS_PER_VERIFY * INT32_OPS_PER_FIELD_OP
# gfx950 full-rate VALU issue: 256 CU x 4 SIMD x 32 lanes/clk x 2.4 GHz
PEAK_INT32_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12
C2_N = 65536


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=C2_N, help="triples per rank")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=1.5, help="wall budget of the CPU sample")
    ap.add_argument("--no-secondary", action="store_true", help="skip the C3/C4 secondary measurements")
    ap.add_argument("--c3-certs", type=int, default=10000, help="C3 certificates per round")
    ap.add_argument("--c4-batches", type=str, default="1024,16384")
    return ap.parse_args()


def cpu_baseline(msgs, pks, sigs, seconds):
    """Oracle (C port of dalek's algorithms) on this host: all threads we may
    use, repeated passes over the workload's first triples until `seconds`."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np

    import coa_oracle

    coa_oracle.build()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count() or 1
    threads = max(1, min(threads, os.cpu_count() or 1, 64))
    chunk = min(len(pks), 4096 * threads)
    m, p, s = msgs[:chunk], pks[:chunk], sigs[:chunk]
    coa_oracle.verify_strict_many(m[:64], p[:64], s[:64], 1)  # table init
    done, t0 = 0, time.perf_counter()
    while True:
        v = coa_oracle.verify_strict_many(m, p, s, threads)
        assert int(v.sum()) == 0, "CPU oracle rejected a valid benchmark signature"
        done += chunk
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    t1 = time.perf_counter()
    one = coa_oracle.verify_strict_many(m[:2048], p[:2048], s[:2048], 1)
    st = time.perf_counter() - t1
    assert int(one.sum()) == 0
    out = {
        "value": done / el,
        "unit": "verifications/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{done} C2 triples ({done // chunk} passes over the first {chunk}) verify_strict, "
                  f"{threads} threads, {el:.1f} s wall ({el * threads:.1f} thread-s)",
        "single_thread_value": 2048 / st,
    }
    out["host"] = host_cpu()
    sodium = libsodium_baseline(m, p, s, threads, min(seconds, 1.0))
    if sodium:
        out["second_reference"] = sodium
    return out


def host_cpu():
    """CPU model and core counts of the box the baseline ran on (SURVEY 8(d):
    report nproc and the CPU model).  `usable_cpus` is this process's
    affinity set; `nproc` the whole machine."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = None
    return {"cpu_model": model, "nproc": os.cpu_count(), "usable_cpus": usable}


def libsodium_baseline(m, p, s, threads, seconds):
    """Second CPU reference: libsodium's
    crypto_sign_verify_detached on the same triples and thread split, driven
    from C threads (oracle/sodium_drive.c), when the box has the library.  Its
    acceptance rules differ from dalek's only on non-canonical and small-order
    encodings, which these valid triples do not contain."""
    import coa_oracle

    first = coa_oracle.sodium_verify_many(m[:64], p[:64], s[:64], 1)
    if first is None:
        return None
    done, t0 = 0, time.perf_counter()
    while True:
        out, ver = coa_oracle.sodium_verify_many(m, p, s, threads)
        assert int(out.sum()) == 0, "libsodium rejected a valid benchmark signature"
        done += len(p)
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    t1 = time.perf_counter()
    one, _ = coa_oracle.sodium_verify_many(m[:2048], p[:2048], s[:2048], 1)
    st = time.perf_counter() - t1
    assert int(one.sum()) == 0
    return {"value": done / el, "unit": "verifications/s", "cores": threads, "single_thread_value": 2048 / st,
            "kind": f"libsodium {ver} crypto_sign_verify_detached",
            "sample": f"{done} C2 triples ({done // len(p)} passes over the first {len(p)}), {threads} threads"}


def worker_batches_on_device(nb, dev):
    """nb bincode WorkerMessage::Batch buffers (977 x 512 B txs, 508,052 B,
    workloads.worker_batch format) built directly in HBM."""
    import torch

    from workloads import TX_SIZE, TXS_PER_BATCH

    rec = 8 + TX_SIZE
    blen = 12 + TXS_PER_BATCH * rec
    data = torch.zeros((nb, blen), dtype=torch.uint8, device=dev)
    data[:, 4] = TXS_PER_BATCH & 0xFF
    data[:, 5] = TXS_PER_BATCH >> 8
    t = torch.arange(TXS_PER_BATCH, device=dev)
    pos = 12 + t * rec
    data[:, pos + 1] = TX_SIZE >> 8  # u64 LE length 512
    data[:, pos + 8] = (t != 0).to(torch.uint8)  # tag: sample tx 0, standard 1
    ctr = torch.arange(nb, device=dev)[:, None] * TXS_PER_BATCH + t[None, :]
    for k in range(8):  # u64 big-endian counter
        data[:, pos + 9 + k] = ((ctr >> (8 * (7 - k))) & 0xFF).to(torch.uint8)
    offs = torch.arange(nb + 1, device=dev, dtype=torch.int64) * blen
    return data.reshape(-1), offs, blen


def c5_shard(local, dev, stream, n=1 << 21, steps=3):
    """One C5 shard per GPU (2^24 triples / 8 GPUs = 2,097,152, BASELINE.json
    configs[4]) as ONE verify call, all valid: the per-GPU rate behind the
    north star's 8-GPU target.  (Its 1 % adversarial parity run is
    tools/c5_parity.py.)"""
    import torch

    import coa_crypto
    import workloads

    seeds = torch.from_numpy(workloads.key_seeds(n)).to(dev)
    msgs = torch.from_numpy(workloads.messages(n)).to(dev)
    pks = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    sigs = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    coa_crypto.sign_many_device(local, seeds, msgs, pks, sigs)
    del seeds
    verdicts = torch.ones(n, dtype=torch.uint8, device=dev)
    ws = torch.empty(coa_crypto.verify_workspace_bytes(n), dtype=torch.uint8, device=dev)
    coa_crypto.verify_strict_many_device(local, msgs, pks, sigs, verdicts, ws, stream)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        coa_crypto.verify_strict_many_device(local, msgs, pks, sigs, verdicts, ws, stream)
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    ok = int(verdicts.sum().item()) == 0
    del msgs, pks, sigs, verdicts, ws
    torch.cuda.empty_cache()
    return {"workload": f"C5 shard: {n:,} triples (2^24 / 8 GPUs) per verify call, all valid",
            "ms_per_call": round(ms, 3), "verifications_per_s": round(n / (ms * 1e-3), 1),
            "frac": round(ALG_INT32_OPS_PER_VERIFY * n / (ms * 1e-3) / 1e12 / PEAK_INT32_TOPS, 4),
            "verdicts_ok": ok}


def batch_alg_int32_ops(n):
    """SURVEY.md 8(d) W_batch(n): 2n decompressions (276 field ops each),
    Pippenger with c = 5 over 2n + 1 (+32) points (9 field ops per addition,
    51 windows) and 253 doublings (8 each), x 200 INT32 ops per field op."""
    return (2 * n * 276 + 9 * 51 * (2 * n + 1 + 32) + 8 * 253) * INT32_OPS_PER_FIELD_OP


def verify_batch_config(local, dev, stream, n_large=1 << 21, n_cert=67, samples=300, cpu_samples=30):
    """Signature::verify_batch (crypto/src/lib.rs:206-219) through the
    Pippenger kernels (csrc/coa_msm.hip), uncached keys:
      large_group       ONE batch equation over n_large signatures resident in
                        HBM (coa_ed25519_verify_batch_device), HIP events;
                        frac against the VALU peak with SURVEY 8(d)'s W_batch
      single_group      one certificate's 67 votes through the host-pointer
                        C ABI (coa_ed25519_verify_batch: H2D + kernels + D2H),
                        p50/p99, beside the C restatement of dalek's
                        verify_batch (Straus, as dalek below 190 points) on
                        one core."""
    import numpy as np
    import torch

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import coa_crypto
    import coa_oracle
    import workloads

    coa_oracle.build()
    out = {}
    n = n_large
    m = torch.from_numpy(np.tile(workloads.messages(1), (n, 1))).to(dev)
    seeds = torch.from_numpy(workloads.key_seeds(n)).to(dev)
    pks = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    sigs = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    coa_crypto.sign_many_device(local, seeds, m, pks, sigs, stream=stream)
    msg = m[0].contiguous()
    del seeds, m
    verdict = torch.ones(1, dtype=torch.uint8, device=dev)
    ws = torch.empty(coa_crypto.verify_batch_workspace_bytes(n), dtype=torch.uint8, device=dev)
    coa_crypto.verify_batch_device(local, msg, pks, sigs, verdict, rng_seed=11, workspace=ws, stream=stream)
    torch.cuda.synchronize()
    steps = 3
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        coa_crypto.verify_batch_device(local, msg, pks, sigs, verdict, rng_seed=11, workspace=ws, stream=stream)
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    out["large_group"] = {
        "workload": f"one verify_batch group of {n:,} signatures (one message), HBM-resident, Pippenger",
        "ms_per_call": round(ms, 3), "signatures_per_s": round(n / (ms * 1e-3), 1),
        "alg_int32_ops": batch_alg_int32_ops(n),
        "frac": round(batch_alg_int32_ops(n) / (ms * 1e-3) / 1e12 / PEAK_INT32_TOPS, 4),
        "verdict_ok": int(verdict.item()) == 0}
    del pks, sigs, ws, verdict
    torch.cuda.empty_cache()

    # one certificate's votes, host pointers (the Rust shim's call)
    mh = workloads.messages(1)
    seeds_h = workloads.key_seeds(n_cert, start=1000)
    pk_h, sg_h = coa_crypto.sign_many(seeds_h, np.tile(mh, (n_cert, 1)))
    offs = np.array([0, n_cert], np.uint64)
    lat = []
    for i in range(samples + 20):
        t0 = time.perf_counter()
        v = coa_crypto.verify_batch_groups(mh, pk_h, sg_h, offs, rng_seed=0)
        lat.append(time.perf_counter() - t0)
        assert int(v[0]) == 0
    lat = np.array(lat[20:]) * 1e3
    rng = np.random.default_rng(5)
    zs = [int.from_bytes(rng.bytes(16), "little") for _ in range(n_cert)]
    pl, sl = [bytes(r) for r in pk_h], [bytes(r) for r in sg_h]
    cl = []
    for _ in range(cpu_samples):
        t0 = time.perf_counter()
        ok = coa_oracle.verify_batch(bytes(mh[0]), pl, sl, zs)
        cl.append(time.perf_counter() - t0)
        assert ok
    cpu_p50 = float(np.percentile(np.array(cl) * 1e3, 50))
    out["single_group"] = {
        "workload": f"verify_batch of one certificate's {n_cert} votes, host pointers in, verdict out",
        "path": "Pippenger (a one-group call routes there at any size)",
        "p50_ms": round(float(np.percentile(lat, 50)), 3), "p99_ms": round(float(np.percentile(lat, 99)), 3),
        "samples": samples,
        "cpu_baseline": {"p50_ms": round(cpu_p50, 3), "cores": 1, "kind": "port",
                         "sample": f"{cpu_samples} calls of the C restatement of dalek verify_batch, single thread"},
        "p50_vs_cpu": round(cpu_p50 / float(np.percentile(lat, 50)), 2)}
    return out


def c4_sha512(local, dev, stream, counts, steps, cpu_threads):
    """C4: SHA-512 Digest over 500 KB worker batches (worker/src/processor.rs:38)."""
    import hashlib

    import numpy as np
    import torch

    import coa_crypto
    import workloads

    out = {"workload": "C4: Sha512 digest of bincode WorkerMessage::Batch (977 x 512 B txs = 508,052 B)"}
    for nb in counts:
        data, offs, blen = worker_batches_on_device(nb, dev)
        dig = torch.empty((nb, 64), dtype=torch.uint8, device=dev)
        coa_crypto.sha512_many_device(local, data, offs, dig, stream)
        torch.cuda.synchronize()
        d = dig.cpu().numpy()
        for b in (0, nb - 1):
            assert bytes(d[b]) == hashlib.sha512(workloads.worker_batch(b)).digest(), "C4 digest mismatch"
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(steps):
            coa_crypto.sha512_many_device(local, data, offs, dig, stream)
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / steps
        out[f"batches_{nb}"] = {"ms_per_launch": round(ms, 3), "GBps": round(nb * blen / (ms * 1e-3) / 1e9, 2),
                                "batches_per_s": round(nb / (ms * 1e-3), 1)}
        del data, dig
        torch.cuda.empty_cache()
    # CPU: the C SHA-512 over host copies, all threads
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import coa_oracle

    nbc = 8 * cpu_threads
    host = np.frombuffer(b"".join(workloads.worker_batch(b) for b in range(nbc)), np.uint8)
    hoffs = np.arange(nbc + 1, dtype=np.uint64) * 508052
    t0 = time.perf_counter()
    coa_oracle.sha512_many(host, hoffs, cpu_threads)
    el = time.perf_counter() - t0
    out["cpu_baseline"] = {"GBps": round(host.size / el / 1e9, 3), "cores": cpu_threads, "kind": "port",
                           "sample": f"{nbc} batches, {cpu_threads} threads"}
    return out


def certificate_config(n_certs, latency_samples, cpu_threads, dev, stream, committee_size=100, n_payload=32):
    """C3 (committee of 100, 67 votes per certificate, 32 payload digests and
    67 parents per header) or C1 (committee of 4, 3 votes, 1 payload digest,
    3 parents): Certificate::verify through the fused path (committee key
    cache f2 + one-launch crypto f3):
      certs_per_s       a round of n_certs certificates resident in HBM,
                        coa_certificate_verify_many_device, HIP events
      host_certs_per_s  the same round through the host-pointer C ABI
                        (PCIe and host packing included)
      p50/p99           one certificate at a time through
                        coa_certificate_verify (host pointers in, verdict out:
                        H2D + kernel + D2H), latency_samples samples
    cpu_baseline: the C restatement of dalek's Certificate::verify crypto on
    one core (the reference verifies certificates serially in Core::run)."""
    import numpy as np
    import torch

    import certificates as C
    import coa_crypto

    committee, batch = C.synth_certificates(n_certs, committee_size=committee_size, n_payload=n_payload, seed=3)
    t0 = time.perf_counter()
    committee.register()
    reg_ms = (time.perf_counter() - t0) * 1e3
    v = C.verify_certificate_batch(batch, committee)  # warm-up + correctness (host path)
    assert int(v.sum()) == 0, "certificates rejected"
    rounds = np.full(n_certs, batch.round, np.uint64)
    t0 = time.perf_counter()
    st = coa_crypto.certificate_verify_many(batch.header_inputs, batch.ids, batch.authors, batch.header_sigs, rounds,
                                            batch.vote_pks, batch.vote_sigs, batch.offsets)
    host_el = time.perf_counter() - t0
    assert int(st.sum()) == 0
    # device-resident round
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a).copy()).to(dev)  # noqa: E731
    hoff = np.zeros(n_certs + 1, np.uint64)
    hoff[1:] = np.cumsum([len(h) for h in batch.header_inputs])
    d = [T(np.frombuffer(b"".join(batch.header_inputs), np.uint8)), T(hoff.view(np.int64)), T(batch.ids),
         T(batch.authors), T(batch.header_sigs), T(rounds.view(np.int64)), T(batch.vote_pks), T(batch.vote_sigs),
         T(batch.offsets.view(np.int64))]
    status = torch.ones(n_certs, dtype=torch.int32, device=dev)
    cws = torch.empty(coa_crypto.certificate_workspace_bytes(n_certs, int(batch.offsets[-1])), dtype=torch.uint8,
                      device=dev)
    coa_crypto.certificate_verify_many_device(0 if dev.index is None else dev.index, *d, status, stream, cws)
    torch.cuda.synchronize()
    assert int(status.abs().sum().item()) == 0, "fused device path rejected certificates"
    reps = 5
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        coa_crypto.certificate_verify_many_device(0 if dev.index is None else dev.index, *d, status, stream, cws)
    e1.record(stream)
    torch.cuda.synchronize()
    dev_ms = e0.elapsed_time(e1) / reps
    del d, status, cws
    # latency: one certificate per call
    lat = []
    for i in range(latency_samples + 20):
        c = i % n_certs
        lo, hi = int(batch.offsets[c]), int(batch.offsets[c + 1])
        args = (batch.header_inputs[c], bytes(batch.ids[c]), bytes(batch.authors[c]), bytes(batch.header_sigs[c]),
                batch.round, batch.vote_pks[lo:hi], batch.vote_sigs[lo:hi])
        t1 = time.perf_counter()
        r = coa_crypto.certificate_verify(*args)
        lat.append(time.perf_counter() - t1)
        assert r == 0
    lat = np.array(lat[20:]) * 1e3
    nv = int(batch.offsets[-1])
    q = committee.quorum_threshold()
    name = "C3" if committee_size == 100 else "C1" if committee_size == 4 else f"committee {committee_size}"
    res = {"workload": f"{name}: committee {committee_size}, {q} votes/certificate, header {n_payload} payload + "
                       f"{q} parents ({len(batch.header_inputs[0]):,} B)",
           "path": "fused: committee key cache + coa_certificate_verify[_many] (one launch)",
           "certificates": n_certs, "votes": nv, "register_ms": round(reg_ms, 2),
           "certs_per_s": round(n_certs / (dev_ms * 1e-3), 1), "round_ms": round(dev_ms, 3),
           "signatures_per_s": round((nv + n_certs) / (dev_ms * 1e-3), 1),
           "host_certs_per_s": round(n_certs / host_el, 1),
           "p50_ms": round(float(np.percentile(lat, 50)), 3), "p99_ms": round(float(np.percentile(lat, 99)), 3),
           "latency_samples": latency_samples}
    # CPU: Certificate::verify crypto (dalek algorithms) on one core
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import random

    import coa_oracle

    rnd = random.Random(1)
    cl = []
    for i in range(min(30, n_certs)):
        lo, hi = int(batch.offsets[i]), int(batch.offsets[i + 1])
        zs = [rnd.getrandbits(128) for _ in range(hi - lo)]
        t1 = time.perf_counter()
        ok = coa_oracle.certificate_verify(batch.header_inputs[i], batch.ids[i], batch.authors[i],
                                           batch.header_sigs[i], batch.round, batch.vote_pks[lo:hi],
                                           batch.vote_sigs[lo:hi], zs)
        cl.append(time.perf_counter() - t1)
        assert ok
    cl = np.array(cl) * 1e3
    res["cpu_baseline"] = {"p50_ms": round(float(np.percentile(cl, 50)), 3), "cores": 1, "kind": "port",
                           "certs_per_s_all_cores_est": round(cpu_threads / (float(np.mean(cl)) * 1e-3), 1),
                           "sample": f"{len(cl)} certificates, single thread"}
    res["p50_vs_cpu"] = round(res["cpu_baseline"]["p50_ms"] / res["p50_ms"], 2)
    return res


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    import coa_crypto
    import sharding
    import workloads

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a HIP device (no CPU fallback)")
    # bind this rank to its GPU before RCCL sees it (one process per GPU)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group(backend="nccl", device_id=dev)
    coa_crypto.init_devices([local])  # this rank's GPU only

    n = args.n
    base, _ = sharding.rank_slice(rank, world, n)  # this rank's contiguous index range
    seeds_h = workloads.key_seeds(n, start=base)
    msgs_h = workloads.messages(n, start=base)
    seeds = torch.from_numpy(seeds_h).to(dev)
    msgs = torch.from_numpy(msgs_h).to(dev)
    pks = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    sigs = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    coa_crypto.sign_many_device(local, seeds, msgs, pks, sigs)
    verdicts = torch.ones(n, dtype=torch.uint8, device=dev)
    ws = torch.empty(coa_crypto.verify_workspace_bytes(n), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()

    # an explicit stream: its handle is never NULL (NULL selects the engine's
    # own stream in the C ABI), so the HIP events below bracket the kernels
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)

    def step(evs=None):
        # one Signature::verify call over the batch: challenge hash, halving,
        # [e]B, decompressions, tables and the joint Horner pass
        if evs is not None:
            evs[0].record(stream)
        coa_crypto.verify_strict_many_device(local, msgs, pks, sigs, verdicts, ws, stream)
        if evs is not None:
            evs[1].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ok = int(verdicts.sum().item()) == 0
    if not ok:
        raise SystemExit("engine rejected valid benchmark signatures")

    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(evs[i])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = sharding.max_over_ranks(elapsed, dist, dev)
    verify_ms = sum(e[0].elapsed_time(e[1]) for e in evs) / args.steps
    ok = ok and int(verdicts.sum().item()) == 0

    total = n * world * args.steps
    value = total / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    achieved = ALG_INT32_OPS_PER_VERIFY * n / (verify_ms * 1e-3) / 1e12
    traffic = None
    tr_path = os.environ.get("COA_TRAFFIC_JSON", os.path.join(ROOT, "profiles", "r01_verify_traffic.json"))
    if os.path.exists(tr_path):
        try:
            with open(tr_path) as f:
                tj = json.load(f)
            if tj.get("n") == n:
                traffic = tj.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(msgs_h, pks.cpu().numpy(), sigs.cpu().numpy(), args.cpu_seconds)
    secondary = None
    if rank == 0 and world == 1 and not args.no_secondary:
        threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count() or 1, 64))
        del ws
        torch.cuda.empty_cache()
        secondary = {
            "c5_shard": c5_shard(local, dev, stream),
            "verify_batch": verify_batch_config(local, dev, stream),
            "c4_sha512": c4_sha512(local, dev, stream, [int(x) for x in args.c4_batches.split(",") if x], 2,
                                   threads),
            "c3_certificate_verify": certificate_config(args.c3_certs, 1000, threads, dev, stream),
            "c1_certificate_verify": certificate_config(2000, 1000, threads, dev, stream, committee_size=4,
                                                        n_payload=1),
        }

    if rank == 0:
        line = {
            "metric": "ed25519 verifications/sec",
            "value": round(value, 1),
            "unit": "verifications/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (seeded RFC 8032 keys/signatures in the reference byte formats, signed on device)",
            "config": {"workload": "C2: 65,536 independent (32 B digest, pk, sig) triples per GPU, all valid, "
                                   "per-signature verify_strict",
                       "triples_per_gpu": n, "parallelism": f"index-range shards x{world}"},
            "kernel_ms": {"verify_call": round(verify_ms, 4)},
            "verdicts_ok": ok,
            "roofline": {"bound": "valu-int32", "achieved": round(achieved, 3), "peak": round(PEAK_INT32_TOPS, 2),
                         "unit": "TOPS", "frac": round(achieved / PEAK_INT32_TOPS, 4), "traffic": traffic,
                         "kernel": "k_pre_halve+k_verify_main (the whole verify call, HIP events on its stream)",
                         "alg_int32_ops_per_verify": ALG_INT32_OPS_PER_VERIFY},
            "cpu_baseline": cpu,
            "secondary": secondary,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
