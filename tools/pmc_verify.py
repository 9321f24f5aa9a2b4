"""Counter profile of bench.py's C2 verify call, for the bench line's
roofline.issue_frac and roofline.traffic (bench.load_pmc).

Reads three rocprofv3 --pmc passes of `bench.py --no-cpu-baseline
--no-secondary` (one counter set per pass, as MI355X_MICROARCH.md prescribes):
  <root>/pmc_SQ          SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES ...
  <root>/pmc_FETCH_SIZE  FETCH_SIZE
  <root>/pmc_WRITE_SIZE  WRITE_SIZE
keeps the dispatches of the given kernels whose grid matches the C2 launch
(n items), takes per-kernel medians over dispatches and writes one JSON with
the sha256 of the kernels' sources and build flags
(bench.verify_kernel_src_sha256; bench.py uses the figures only while those
are unchanged).  FETCH_SIZE/WRITE_SIZE are KiB; FETCH_SIZE is doubled (the
gfx950 calibration for wide coalesced reads).

usage: python tools/pmc_verify.py <root> <n> <out.json> [kernel ...]
       (default kernels: k_pre_halve k_verify_main)"""
import collections
import csv
import glob
import hashlib
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "xrpl-coa-prototype_amd", "lib", "libcoa_verify.so")


def rows(root, sub):
    for path in glob.glob(os.path.join(root, sub, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            yield from csv.DictReader(f)


def per_dispatch(root, sub, kernels):
    """{kernel: {dispatch: {counter: value}}} plus each dispatch's grid size."""
    out = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    grid = {}
    for r in rows(root, sub):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].strip()
        if k not in kernels:
            continue
        out[k][r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        grid[(k, r["Dispatch_Id"])] = int(r["Grid_Size"])
    return out, grid


def main():
    root, n, dst = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    kernels = sys.argv[4:] or ["k_pre_halve", "k_verify_main"]
    sys.path.insert(0, ROOT)
    import bench

    res = {"n": n, "kernels": {}, "lib_sha256": hashlib.sha256(open(LIB, "rb").read()).hexdigest(),
           "kernel_src_sha256": bench.verify_kernel_src_sha256(),
           "command": "rocprofv3 --pmc <set> -- python3 bench.py --no-cpu-baseline --no-secondary --steps 3 "
                      "--warmup 1 (one pass per counter set)",
           "note": "medians over dispatches of the C2 launch; SQ_WAVE_CYCLES in quad-cycles (x4); FETCH_SIZE "
                   "doubled per the gfx950 calibration; per-launch totals"}
    sq, grid = per_dispatch(root, "pmc_SQ", kernels)
    fe, _ = per_dispatch(root, "pmc_FETCH_SIZE", kernels)
    wr, _ = per_dispatch(root, "pmc_WRITE_SIZE", kernels)
    valu = fetch = write = 0.0
    for k in kernels:
        if k not in sq:
            raise SystemExit(f"no SQ rows for {k} under {root}")
        # the C2 launch is the most frequent grid size among this kernel's dispatches
        sizes = collections.Counter(grid[(k, d)] for d in sq[k])
        g = sizes.most_common(1)[0][0]
        ds = [d for d in sq[k] if grid[(k, d)] == g]
        med = lambda c: statistics.median(sq[k][d].get(c, 0.0) for d in ds)  # noqa: E731
        kv = {"grid": g, "dispatches": len(ds), "waves": med("SQ_WAVES"), "valu_insts": med("SQ_INSTS_VALU"),
              "salu_insts": med("SQ_INSTS_SALU"), "wave_cycles": 4 * med("SQ_WAVE_CYCLES"),
              "busy_cycles": med("SQ_BUSY_CYCLES"), "wait_inst_any": med("SQ_WAIT_INST_ANY"),
              "active_inst_valu": med("SQ_ACTIVE_INST_VALU")}
        kv["valu_insts_per_wave"] = kv["valu_insts"] / max(kv["waves"], 1.0)
        kv["cycles_per_valu_inst"] = kv["wave_cycles"] / max(kv["valu_insts"], 1.0)
        kv["valu_issue_share"] = 2 * kv["valu_insts"] / max(kv["wave_cycles"], 1.0)
        # fraction of the waves' lifetime spent issuing VALU (both counters in quad-cycles)
        kv["valu_active_share"] = kv["active_inst_valu"] * 4 / max(kv["wave_cycles"], 1.0)
        f = [v["FETCH_SIZE"] for v in fe.get(k, {}).values()]
        w = [v["WRITE_SIZE"] for v in wr.get(k, {}).values()]
        if f and w:
            kv["hbm_read_bytes"] = 2 * 1024 * statistics.median(f)
            kv["hbm_write_bytes"] = 1024 * statistics.median(w)
            fetch += kv["hbm_read_bytes"]
            write += kv["hbm_write_bytes"]
        valu += kv["valu_insts"]
        res["kernels"][k] = kv
    res["valu_insts_per_call"] = valu
    tot_cyc = sum(v["wave_cycles"] for v in res["kernels"].values())
    res["valu_active_share"] = (sum(v["active_inst_valu"] * 4 for v in res["kernels"].values()) / tot_cyc
                                if tot_cyc else None)
    res["hbm_bytes_per_launch"] = fetch + write if fetch else None
    res["alg_bytes_per_launch"] = n * (32 + 32 + 64 + 1)
    os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
    with open(dst, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
