#!/bin/bash
# Pippenger bucket phase: run-length A/B (COA_MSM_RUN) on a 2^21 group, kernel
# trace per setting, plus one SQ counter pass of the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
for run in ${RUNS:-128 64 32}; do
  COA_MSM_RUN=$run timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/msm_run$run -o run --output-format csv \
    -- python3 tools/msm_probe.py 2097152 > gpurun_out/msm_run$run.log 2>&1 || exit 1
  echo "run $run: $(tail -1 gpurun_out/msm_run$run.log)"
  python3 - $run <<'PY'
import csv,glob,sys
f=glob.glob(f'gpurun_out/msm_run{sys.argv[1]}/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'msm' in r['Name']: print('  ', r['Name'].split('(')[0], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg')
PY
done
timeout -k 10 -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD \
  -d gpurun_out/msm_pmc -o run --output-format csv -- python3 tools/msm_probe.py 2097152 > gpurun_out/msm_pmc.log 2>&1 || exit 1
python3 - <<'PY'
import csv,glob,collections
acc=collections.defaultdict(lambda: collections.defaultdict(float)); n=collections.Counter()
for f in glob.glob('gpurun_out/msm_pmc/**/*counter_collection.csv',recursive=True):
    for r in csv.DictReader(open(f)):
        k=r['Kernel_Name'].split('(')[0]
        if 'msm' not in k: continue
        acc[k][r['Counter_Name']]+=float(r['Counter_Value'])
for k,v in acc.items():
    wc=4*v['SQ_WAVE_CYCLES']
    print(k, {c: int(x) for c,x in v.items()}, 'valu/wave', round(v['SQ_INSTS_VALU']/max(v['SQ_WAVES'],1)), 'wait_any_share', round(4*v['SQ_WAIT_ANY']/max(wc,1),3), 'active_valu_share', round(v['SQ_ACTIVE_INST_VALU']/max(v['SQ_WAVE_CYCLES'],1)/4,3) if False else round(4*v['SQ_ACTIVE_INST_VALU']/max(wc,1),3))
PY
