"""Per-kernel counter summary of a bench section (SHA-512, Pippenger, ...):
VALU issue against the SIMD's issue peak, active / waiting shares, cycles
per VALU instruction per wave, and traffic per dispatch.

Reads rocprofv3 --pmc passes of one command (one counter set per pass, as
MI355X_MICROARCH.md prescribes; tools/gpu_session.sh pmcsec runs them):
  <root>/pmc_SQ     SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES
                    SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
  <root>/pmc_WAIT   SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INST_CYCLES_VMEM
                    SQ_ACTIVE_INST_ANY SQ_INSTS_LDS
  <root>/pmc_FETCH_SIZE, <root>/pmc_WRITE_SIZE
and the kernel trace of the same passes (durations).  Groups dispatches by
(kernel, grid size) and takes medians.  Derived, per dispatch:
  issue_frac     SQ_INSTS_VALU x 2 cycles / (1,024 SIMDs x 2.4 GHz x duration)
                 -- the share of the chip's VALU issue slots the kernel used
  cycles_per_valu  SQ_WAVE_CYCLES x 4 / SQ_INSTS_VALU (per wave, quad-cycles)
  valu_active_share  SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES
  wait_any_share / vmem_share   SQ_WAIT_ANY, SQ_INST_CYCLES_VMEM / SQ_WAVE_CYCLES
  fetch_bytes / write_bytes     FETCH_SIZE x 2 (gfx950 calibration) and
                 WRITE_SIZE, KiB -> bytes
usage: python tools/pmc_kernels.py <root> <out.json> <kernel> [kernel ...]
       python tools/pmc_kernels.py --raw <root> <out.json>   (every counter of
       every pass directory, medians per (kernel, grid), dispatches with a
       grid of at least 20,000 work-items)"""
import collections
import csv
import glob
import json
import os
import statistics
import sys

SIMDS, CLOCK = 1024, 2.4e9


def _rows(root, sub, suffix):
    for path in glob.glob(os.path.join(root, sub, "**", f"*{suffix}"), recursive=True):
        with open(path) as f:
            yield from csv.DictReader(f)


def _name(s):
    return s.split("(")[0].replace("void ", "").split("<")[0].strip()


def counters(root, sub, kernels):
    """{(kernel, grid): {dispatch: {counter: value}}}"""
    out = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    for r in _rows(root, sub, "counter_collection.csv"):
        k = _name(r["Kernel_Name"])
        if k in kernels:
            out[(k, int(r["Grid_Size"]))][r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    return out


def durations(root, kernels):
    """{(kernel, grid): [ns]} from the kernel traces of every pass."""
    out = collections.defaultdict(list)
    for r in _rows(root, "", "kernel_trace.csv"):
        k = _name(r["Kernel_Name"])
        if k in kernels:
            grid = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
            out[(k, grid)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return out


def raw(root, dst):
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        with open(path) as f:
            for r in csv.DictReader(f):
                g = int(r["Grid_Size"])
                if g >= 20000:
                    per[(_name(r["Kernel_Name"]), g, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        for (k, g, _), cs in per.items():
            for c, v in cs.items():
                out[f"{k}@{g}"][c].append(v)
    res = {k: {c: statistics.median(v) for c, v in cs.items()} for k, cs in out.items()}
    with open(dst, "w") as fh:
        json.dump(res, fh, indent=1)
    for k, cs in sorted(res.items()):
        print(k, {c: round(v, 1) for c, v in sorted(cs.items())})


def main():
    if sys.argv[1] == "--raw":
        raw(sys.argv[2], sys.argv[3])
        return
    root, dst, kernels = sys.argv[1], sys.argv[2], set(sys.argv[3:])
    sq = counters(root, "pmc_SQ", kernels)
    wt = counters(root, "pmc_WAIT", kernels)
    fe = counters(root, "pmc_FETCH_SIZE", kernels)
    wr = counters(root, "pmc_WRITE_SIZE", kernels)
    dur = durations(root, kernels)
    res = {"root": root, "kernels": {}}
    for key in sorted(set(sq) | set(wt) | set(fe)):
        k, grid = key
        med = lambda d, c: statistics.median([v.get(c, 0.0) for v in d[key].values()]) if d.get(key) else None  # noqa
        e = {"grid": grid, "dispatches": len(sq.get(key, {}))}
        ns = statistics.median(dur[key]) if dur.get(key) else None
        e["duration_us"] = ns / 1e3 if ns else None
        valu, cyc = med(sq, "SQ_INSTS_VALU"), med(sq, "SQ_WAVE_CYCLES")
        waves = med(sq, "SQ_WAVES")
        e.update({"waves": waves, "valu_insts": valu, "valu_insts_per_wave": valu / waves if valu and waves else None})
        if valu and ns:
            e["issue_frac"] = valu * 2 / (SIMDS * CLOCK * ns * 1e-9)
        if valu and cyc:
            e["cycles_per_valu_per_wave"] = cyc * 4 / valu
            e["valu_active_share"] = med(sq, "SQ_ACTIVE_INST_VALU") / cyc
            e["wait_inst_any_share"] = med(sq, "SQ_WAIT_INST_ANY") / cyc
        wcyc = med(wt, "SQ_WAVE_CYCLES")
        if wcyc:
            e["wait_any_share"] = med(wt, "SQ_WAIT_ANY") / wcyc
            e["vmem_share"] = med(wt, "SQ_INST_CYCLES_VMEM") / wcyc
            e["active_any_share"] = med(wt, "SQ_ACTIVE_INST_ANY") / wcyc
            e["lds_insts"] = med(wt, "SQ_INSTS_LDS")
        f = med(fe, "FETCH_SIZE")
        w = med(wr, "WRITE_SIZE")
        e["fetch_bytes"] = f * 1024 * 2 if f is not None else None
        e["write_bytes"] = w * 1024 if w is not None else None
        res["kernels"][f"{k}@{grid}"] = e
    with open(dst, "w") as fh:
        json.dump(res, fh, indent=1)
    for name, e in res["kernels"].items():
        print(name, {k: (round(v, 4) if isinstance(v, float) else v) for k, v in e.items()
                     if k in ("duration_us", "issue_frac", "cycles_per_valu_per_wave", "valu_active_share",
                              "wait_any_share", "vmem_share", "fetch_bytes")})


if __name__ == "__main__":
    main()
