"""Per-wave phase stamps (clock64) of the one-wave C2 main kernel
(k_verify_main<1, true>), from a build with -DCOA_MAIN_TRACE: where a lone
wave's time goes between the prologue loads, the digit loop and the [e]B /
identity tail.

  python tools/main_trace.py build   (CPU: build/main_trace/libcoa_verify.so)
  python tools/main_trace.py run     (GPU: C2 calls, prints the phase shares)

Marks: 0 kernel entry, 1 after the prologue loads and the wave's digit
count (wave_max), 2 after the digit loop, 3 after the verdict store."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "xrpl-coa-prototype_amd")
OUT = os.path.join(ROOT, "build", "main_trace")


def build():
    sys.path.insert(0, PKG)
    import build as b

    b.build()
    os.makedirs(OUT, exist_ok=True)
    obj = os.path.join(OUT, "coa_halved.o")
    subprocess.run([b.HIPCC] + b.COMMON + ["-DCOA_MAIN_TRACE", "-c", os.path.join(b.CSRC, "coa_halved.hip"), "-o", obj],
                   check=True)
    objs = [obj if s == "coa_halved.hip" else os.path.join(b.OBJDIR, s + ".o") for s in b.SOURCES]
    subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o", os.path.join(OUT, "libcoa_verify.so")]
                   + objs, check=True)


def run():
    os.environ["COA_VERIFY_LIB"] = os.path.join(OUT, "libcoa_verify.so")
    sys.path.insert(0, PKG)
    import ctypes

    import numpy as np
    import torch

    import coa_crypto
    import workloads

    coa_crypto.init(1)
    n = 65536
    dev = torch.device("cuda", 0)
    seeds = torch.from_numpy(workloads.key_seeds(n)).to(dev)
    m = torch.from_numpy(workloads.messages(n)).to(dev)
    pk = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    sg = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    coa_crypto.sign_many_device(0, seeds, m, pk, sg)
    out = torch.ones(n, dtype=torch.uint8, device=dev)
    f = coa_crypto.lib().coa_main_trace
    f.argtypes = [ctypes.c_void_p]
    for rep in range(30):
        coa_crypto.verify_strict_many_device(0, m, pk, sg, out)
    torch.cuda.synchronize()
    assert int(out.sum().item()) == 0
    for rep in range(3):
        coa_crypto.verify_strict_many_device(0, m, pk, sg, out)
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * (4096 * 4))()
        f(ctypes.addressof(buf))
        t = np.array(list(buf), np.int64).reshape(4096, 4)[: n // 64]
        d = np.diff(t, axis=1).astype(np.float64)
        tot = (t[:, 3] - t[:, 0]).astype(np.float64)
        print(json.dumps({"rep": rep, "waves": int(len(t)),
                          "cycles_per_wave_median": float(np.median(tot)),
                          "prologue_share": round(float(np.median(d[:, 0] / tot)), 4),
                          "loop_share": round(float(np.median(d[:, 1] / tot)), 4),
                          "tail_share": round(float(np.median(d[:, 2] / tot)), 4),
                          "prologue_cycles_p50_p99": [float(np.percentile(d[:, 0], 50)), float(np.percentile(d[:, 0], 99))],
                          "tail_cycles_p50_p99": [float(np.percentile(d[:, 2], 50)), float(np.percentile(d[:, 2], 99))],
                          "wave_start_spread_cycles": float(t[:, 0].max() - t[:, 0].min())}), flush=True)


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
