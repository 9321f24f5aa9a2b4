"""Per-(kernel, grid size) duration summary of a rocprofv3 --kernel-trace run
(kernel_trace.csv), so the C2 dispatches of a full `python bench.py` run can
be told apart from the secondary configurations' launches of the same
kernels.

usage: python tools/kernel_trace_summary.py <dir with *kernel_trace.csv> [out.json]
Prints one line per (kernel, grid) sorted by total time; with out.json also
writes them as JSON."""
import collections
import csv
import glob
import json
import os
import statistics
import sys


def main():
    root = sys.argv[1]
    dur = collections.defaultdict(list)
    for path in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                k = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
                g = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
                dur[(k, g)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = []
    for (k, g), d in dur.items():
        out.append({"kernel": k, "grid": g, "calls": len(d), "total_us": round(sum(d), 1),
                    "avg_us": round(statistics.mean(d), 2), "median_us": round(statistics.median(d), 2),
                    "min_us": round(min(d), 2), "max_us": round(max(d), 2)})
    out.sort(key=lambda x: -x["total_us"])
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            json.dump(out, f, indent=1)
    for o in out:
        print(f"{o['kernel'][:60]:60s} grid {o['grid']:>10d} calls {o['calls']:>5d} avg {o['avg_us']:>10.2f} us "
              f"median {o['median_us']:>10.2f} total {o['total_us']:>12.1f}")


if __name__ == "__main__":
    main()
