"""Build the gfx950 engine library in-tree: xrpl-coa-prototype_amd/lib/libcoa_verify.so.

hipcc cross-compiles for gfx950 without a GPU.  Each translation unit is
compiled separately (in parallel) and only when its sources changed, then
linked into one shared library exporting the C ABI of include/coa_verify.h.
"""
import concurrent.futures
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "lib")
OBJDIR = os.path.join(LIBDIR, "obj")
LIB = os.path.join(LIBDIR, "libcoa_verify.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

SOURCES = ["coa_kernels.hip", "coa_halved.hip", "coa_batch.hip", "coa_committee.hip", "coa_msm.hip", "coa_latency.hip",
           "coa_runtime.cpp", "coa_queue.cpp", "coa_queue_hip.cpp", "coa_wire.cpp", "coa_cpu.cpp"]
HEADERS = ["coa_fe.h", "coa_sc.h", "coa_ge.h", "coa_sha512.h", "coa_smul.h", "coa_kernels.h", "coa_batch.h", "coa_halved.h",
           "coa_committee.h", "coa_msm.h", "coa_fe_wave.h", "coa_ge_rows.h", "coa_halve.h", "coa_keycache.h",
           "coa_latency.h", "coa_queue.h", "coa_rcmp.h", "coa_lehmer.h"]
COMMON = ["-O3", "-fPIC", "-std=c++17", "-ffunction-sections", f"--offload-arch={ARCH}", "-I" + os.path.join(ROOT, "include")]


def _newest(paths):
    return max(os.path.getmtime(p) for p in paths if os.path.exists(p))


def _compile(src):
    path = os.path.join(CSRC, src)
    obj = os.path.join(OBJDIR, src + ".o")
    deps = [path] + [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(ROOT, "include", "coa_verify.h")]
    if os.path.exists(obj) and os.path.getmtime(obj) >= _newest(deps):
        return obj, False
    cmd = [HIPCC] + COMMON + ["-c", path, "-o", obj]
    if src.endswith(".cpp"):
        cmd = [HIPCC, "-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-I" + os.path.join(ROOT, "include"), "-c",
                   path, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-6000:]}")
    return obj, True


def build(verbose=False):
    """Compile (incrementally) and link; returns the library path."""
    os.makedirs(OBJDIR, exist_ok=True)
    with concurrent.futures.ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
        results = list(ex.map(_compile, SOURCES))
    objs = [o for o, _ in results]
    rebuilt = any(b for _, b in results)
    if rebuilt or not os.path.exists(LIB) or os.path.getmtime(LIB) < _newest(objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-pthread", "-o", LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
        if verbose:
            print("built", LIB)
    _build_latc()
    return LIB


def _build_latc():
    """lib/liblatc.so: the C-caller latency loop of tools/latc.c (measurement
    only; bench.py loads it), linked against the engine library."""
    src = os.path.join(ROOT, "tools", "latc.c")
    out = os.path.join(LIBDIR, "liblatc.so")
    if not os.path.exists(src):
        return
    if os.path.exists(out) and os.path.getmtime(out) >= _newest([src, LIB, os.path.join(ROOT, "include", "coa_verify.h")]):
        return
    cmd = ["gcc", "-O2", "-std=c11", "-shared", "-fPIC", "-pthread", "-I" + os.path.join(ROOT, "include"), src, "-o", out,
           "-L" + LIBDIR, "-lcoa_verify", "-Wl,-rpath,$ORIGIN"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"liblatc build failed:\n{r.stderr[-3000:]}")


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
