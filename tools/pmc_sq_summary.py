"""Per-wave SQ figures of selected kernels from a rocprofv3 --pmc pass
(counter_collection.csv), medians over dispatches.

usage: python tools/pmc_sq_summary.py <counter_collection.csv> <kernel> [<kernel> ...]

SQ_WAVE_CYCLES and SQ_WAIT_INST_ANY count quad-cycles (MI355X_MICROARCH.md),
so per-wave cycles are x4.  "VALU issue share" = VALU instructions x 2 cycles
(the full-rate issue cost of a wave64 VALU instruction on one SIMD) over the
wave's cycles: 1.0 would be one VALU instruction every 2 cycles for the
wave's whole life."""
import collections
import csv
import statistics
import sys


def main():
    path, kernels = sys.argv[1], sys.argv[2:]
    per = collections.defaultdict(lambda: collections.defaultdict(float))  # (kernel, dispatch) -> counter
    meta = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            k = row["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
            if k not in kernels:
                continue
            key = (k, row["Dispatch_Id"])
            per[key][row["Counter_Name"]] += float(row["Counter_Value"])
            meta[k] = (row["Grid_Size"], row["Workgroup_Size"], row["VGPR_Count"], row["Scratch_Size"])
    for k in kernels:
        rows = [c for (kk, _), c in per.items() if kk == k]
        if not rows:
            continue

        def med(fn):
            return statistics.median(fn(c) for c in rows)

        waves = med(lambda c: c["SQ_WAVES"])
        valu = med(lambda c: c["SQ_INSTS_VALU"] / c["SQ_WAVES"])
        salu = med(lambda c: c["SQ_INSTS_SALU"] / c["SQ_WAVES"])
        vmem = med(lambda c: c.get("SQ_INSTS_VMEM", 0.0) / c["SQ_WAVES"])
        cyc = med(lambda c: 4 * c["SQ_WAVE_CYCLES"] / c["SQ_WAVES"])
        wait = med(lambda c: c["SQ_WAIT_INST_ANY"] / max(c["SQ_WAVE_CYCLES"], 1.0))
        g, wg, vgpr, scr = meta[k]
        print(f"{k}: dispatches {len(rows)}  grid {g}  wg {wg}  vgpr {vgpr}  scratch {scr}  waves {waves:,.0f}  "
              f"VALU instr/wave {valu:,.0f}  SALU instr/wave {salu:,.0f}  VMEM instr/wave {vmem:,.1f}  "
              f"cycles/wave {cyc:,.0f}  cycles per VALU instr {cyc / valu:.2f}  "
              f"VALU issue share {2 * valu / cyc:.3f}  wait share {wait:.2%}")


if __name__ == "__main__":
    main()
