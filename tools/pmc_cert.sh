#!/bin/bash
# PMC SQ counters of the Certificate::verify throughput kernel (k_cert_verify)
# over a C3 round (tools/cert_probe.py 10000), per wave; kernel trace stats
# in a separate pass.  Run on the GPU box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU -d gpurun_out/pmc_cert -o run --output-format csv -- python3 tools/cert_probe.py 10000 > gpurun_out/pmc_cert.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cert -o run --output-format csv -- python3 tools/cert_probe.py 10000 > gpurun_out/prof_cert.log 2>&1 || exit 1
f=$(find gpurun_out/pmc_cert -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in rows:
    k = r["Kernel_Name"].split("(")[0]
    if not k.startswith("k_cert") and not k.startswith("k_sha") and not k.startswith("k_batch"):
        continue
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r.get("Dispatch_Id"))
for k, v in agg.items():
    w = v["SQ_WAVES"]
    print(k, "dispatches", len(disp[k]), {c: round(x / w, 1) for c, x in v.items() if c != "SQ_WAVES"},
          "waves", int(w), "| wait_any/wave_cycles", round(v["SQ_WAIT_ANY"] / v["SQ_WAVE_CYCLES"], 3),
          "| wait_inst/wave_cycles", round(v["SQ_WAIT_INST_ANY"] / v["SQ_WAVE_CYCLES"], 3),
          "| quad-cycles per VALU", round(v["SQ_WAVE_CYCLES"] / v["SQ_INSTS_VALU"], 2))
PY
for f in $(find gpurun_out/prof_cert -name "*kernel_stats.csv"); do head -8 "$f"; done
