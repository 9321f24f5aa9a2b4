"""Median duration per (kernel, grid) from the kernel traces that
tools/gpu_session.sh kstats TAG leaves under gpurun_out/kstats_TAG, plus the
bench line's verify_batch large-group figure.
usage: python tools/kstats_grid.py SUBSTRING MIN_GRID TAG [TAG ...]"""
import collections
import csv
import glob
import json
import sys


def main():
    sub, min_grid, tags = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
    for t in tags:
        d = collections.defaultdict(list)
        for f in glob.glob(f"gpurun_out/kstats_{t}/**/*kernel_trace.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                n = r["Kernel_Name"]
                g = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
                if sub in n and g >= min_grid:
                    d[(n.split("(")[0].replace("void ", ""), g)].append(
                        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        extra = ""
        try:
            for line in open(f"gpurun_out/kstats_{t}.json"):
                if line.startswith("{"):
                    lg = json.loads(line).get("secondary", {}).get("verify_batch", {}).get("large_group")
                    if lg:
                        extra = f" ms_per_call={lg['ms_per_call']} frac={lg['frac']}"
        except OSError:
            pass
        print(t, {f"{k}@{g}": round(sorted(v)[len(v) // 2], 1) for (k, g), v in sorted(d.items())}, extra)


if __name__ == "__main__":
    main()
