"""SQ issue/wait shares of the C2 verify kernels from a tools/pmc_wait.sh pass
(rocprofv3 counter CSV) -> JSON: medians over dispatches, shares of
SQ_WAVE_CYCLES (quad-cycles)."""
import collections
import csv
import json
import sys


def main(csv_path, out_path, note):
    rows = list(csv.DictReader(open(csv_path)))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in rows:
        k = r["Kernel_Name"]
        for name in ("k_verify_main", "k_pre_halve"):
            if name in k and r["Grid_Size"] in ("65536", "196608"):
                agg[name][(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    out = {"command": "tools/pmc_wait.sh (rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY "
                      "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INSTS_BRANCH -- "
                      "python3 bench.py --no-cpu-baseline --no-secondary --steps 3 --warmup 1)",
           "note": note, "kernels": {}}
    for name, d in agg.items():
        per = collections.defaultdict(list)
        for (_, c), v in d.items():
            per[c].append(v)
        med = {c: sorted(v)[len(v) // 2] for c, v in per.items()}
        wc = med["SQ_WAVE_CYCLES"]
        out["kernels"][name] = {**med, "active_any_share": round(med["SQ_ACTIVE_INST_ANY"] / wc, 4),
                                "active_valu_share": round(med["SQ_ACTIVE_INST_VALU"] / wc, 4),
                                "wait_any_share": round(med["SQ_WAIT_ANY"] / wc, 4)}
    json.dump(out, open(out_path, "w"), indent=1)
    for k, v in out["kernels"].items():
        print(k, v["active_any_share"], v["active_valu_share"], v["wait_any_share"])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "")
