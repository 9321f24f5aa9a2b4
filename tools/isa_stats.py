"""Static ISA statistics of a HIP translation unit for gfx950.

Compiles with -save-temps into a temp dir and reports per kernel: instruction
count, s_nop count, v_mad_u64_u32 / v_mov counts, VGPRs, spilled VGPRs and
private segment bytes.  Used to audit hipcc's hazard pads and register
pressure ("Field arithmetic").

usage: python tools/isa_stats.py SRC.hip [-DNAME=VAL ...]
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def stats(src, defines=()):
    with tempfile.TemporaryDirectory() as d:
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffunction-sections", "-I" + os.path.join(ROOT, "include"),
               "-c", os.path.abspath(src), "-save-temps", "-o", os.path.join(d, "x.o")] + list(defines)
        subprocess.run(cmd, cwd=d, check=True, capture_output=True)
        base = os.path.splitext(os.path.basename(src))[0]
        s = open(os.path.join(d, f"{base}-hip-amdgcn-amd-amdhsa-gfx950.s")).read()
    out = {}
    for name in re.findall(r"^(_Z\w+):", s, re.M):
        i = s.index(name + ":")
        j = s.find(".Lfunc_end", i)
        if j < 0:
            continue
        body = s[i:j].split("\n")
        ins = [l.strip().split()[0] for l in body
               if l.startswith("\t") and l.strip() and not l.startswith("\t.") and not l.startswith("\t;")]
        c = collections.Counter(ins)
        out[name] = dict(instrs=len(ins), s_nop=c["s_nop"], mad=c["v_mad_u64_u32"], mov=c["v_mov_b32_e32"])
    # metadata: one YAML entry per kernel, keys sorted; .name precedes the counts we want
    for ent in re.split(r"\n  - \.agpr_count:", s)[1:]:
        m = re.search(r"\.name:\s+(\S+)", ent)
        if not m or m.group(1) not in out:
            continue
        for key in ("vgpr_count", "vgpr_spill_count", "private_segment_fixed_size"):
            mm = re.search(r"\." + key + r":\s+(\d+)", ent)
            out[m.group(1)][key] = int(mm.group(1)) if mm else None
    return out


if __name__ == "__main__":
    for k, v in stats(sys.argv[1], sys.argv[2:]).items():
        print(f"{k[:48]:48s} " + " ".join(f"{a}={b}" for a, b in v.items()))
