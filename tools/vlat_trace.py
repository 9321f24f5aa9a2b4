"""Phase timestamps (clock64 ticks, 100 MHz on gfx950... read as relative
units) of the single-signature latency kernel k_verify_lat, from a build with
-DCOA_VLAT_TRACE.

  python tools/vlat_trace.py build   (CPU: writes build/vlat_trace/libcoa_verify.so)
  python tools/vlat_trace.py run     (GPU: one uncached and one cached verify)

Marks per wave: 0 start, 1 phase-1 work done (hash/halving, decompression +
table, comb butterflies), 2 after the first barrier, 3 phase-2 work done
(Horner chains, [e]B), 4 after the second barrier, 5 verdict (wave 0)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "xrpl-coa-prototype_amd")
OUT = os.path.join(ROOT, "build", "vlat_trace")


def build():
    sys.path.insert(0, PKG)
    import build as b

    b.build()
    os.makedirs(OUT, exist_ok=True)
    obj = os.path.join(OUT, "coa_latency.o")
    subprocess.run([b.HIPCC] + b.COMMON + ["-DCOA_VLAT_TRACE", "-c", os.path.join(b.CSRC, "coa_latency.hip"), "-o",
                                           obj], check=True)
    objs = [obj if s == "coa_latency.hip" else os.path.join(b.OBJDIR, s + ".o") for s in b.SOURCES]
    subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-pthread", "-o",
                    os.path.join(OUT, "libcoa_verify.so")] + objs, check=True)


def run():
    os.environ["COA_VERIFY_LIB"] = os.path.join(OUT, "libcoa_verify.so")
    sys.path.insert(0, PKG)
    import ctypes

    import numpy as np
    import torch  # noqa: F401

    import coa_crypto
    from workloads import key_seeds, messages

    coa_crypto.init(1)
    pks, sigs = coa_crypto.sign_many(key_seeds(4, 11), messages(4, 11))
    msgs = messages(4, 11)
    f = coa_crypto.lib().coa_vlat_trace
    f.argtypes = [ctypes.c_void_p]
    for label, reg in (("uncached", False), ("cached", True)):
        coa_crypto.committee_register(pks if reg else np.zeros((0, 32), np.uint8))
        for rep in range(4):
            v = coa_crypto.verify_strict_many(msgs[:1], pks[:1], sigs[:1])
            assert int(v[0]) == 0
            buf = (ctypes.c_ulonglong * 32)()
            f(ctypes.addressof(buf))
            t = np.array(list(buf), np.int64).reshape(4, 8)
            t0 = t[:, 0].min()
            print(json.dumps({"path": label, "rep": rep, **{f"wave{w}": (t[w, :6] - t0).tolist() for w in range(4)}}),
                  flush=True)


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
