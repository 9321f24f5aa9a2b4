"""Build a variant of the engine library with extra preprocessor defines into
build/<name>/libcoa_verify.so, for same-box A/B runs through COA_VERIFY_LIB
(bench.py and coa_crypto load that path).  Measurement infrastructure only.

usage: python tools/build_variant.py <name> -DNAME=VALUE [...]
e.g.   python tools/build_variant.py w26 -DCOA_WCOMB_W=26 -DCOA_WCOMB_POS=10"""
import concurrent.futures
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xrpl-coa-prototype_amd"))
import build as B  # noqa: E402


def main():
    name, defines = sys.argv[1], sys.argv[2:]
    out = os.path.join(ROOT, "build", name)
    os.makedirs(out, exist_ok=True)

    def one(src):
        obj = os.path.join(out, src + ".o")
        flags = B.COMMON if src.endswith(".hip") else ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={B.ARCH}",
                                                        "-I" + os.path.join(ROOT, "include")]
        r = subprocess.run([B.HIPCC] + flags + defines + ["-c", os.path.join(B.CSRC, src), "-o", obj],
                           capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError(f"{src}: {r.stderr[-4000:]}")
        return obj

    with concurrent.futures.ThreadPoolExecutor(max_workers=len(B.SOURCES)) as ex:
        objs = list(ex.map(one, B.SOURCES))
    lib = os.path.join(out, "libcoa_verify.so")
    r = subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-pthread", "-o", lib] + objs,
                       capture_output=True, text=True)
    if r.returncode:
        raise RuntimeError(r.stderr[-4000:])
    for o in objs:
        os.remove(o)
    # the C-caller loop bench.py times, bound to this build through $ORIGIN
    latc = os.path.join(out, "liblatc.so")
    r = subprocess.run(["gcc", "-O2", "-std=c11", "-shared", "-fPIC", "-pthread", "-I" + os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "tools", "latc.c"), "-o", latc, "-L" + out, "-lcoa_verify",
                        "-Wl,-rpath,$ORIGIN"], capture_output=True, text=True)
    if r.returncode:
        raise RuntimeError(r.stderr[-4000:])
    print(lib)


if __name__ == "__main__":
    main()
