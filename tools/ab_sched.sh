#!/bin/bash
# Kernel-time A/B of two library builds under rocprofv3 --kernel-trace --stats
# (k_verify_main / k_pre_halve average and minimum over a 40-step C2 bench);
# round 2 compared a build of coa_halved.hip with -mllvm
# -amdgpu-sched-strategy=max-ilp (build/ab/libcoa_verify_ilp.so) against the default.
cd "${GRAFT_REPO_ROOT}" && export TMPDIR=/tmp && mkdir -p gpurun_out
for kv in ilp=build/ab/libcoa_verify_ilp.so head=build/ab/libcoa_verify_head.so; do
  name=${kv%%=*}; lib=${kv#*=}
  COA_VERIFY_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/sched_$name -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-secondary --steps 40 > gpurun_out/sched_$name.json 2>/dev/null || exit 1
  python3 -c "
import csv,glob
f=glob.glob('gpurun_out/sched_$name/**/run_kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'verify_main' in r['Name'] or 'pre_halve' in r['Name']: print('$name', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,1), round(float(r['MinNs'])/1e3,1))
import json; print('$name value', json.load(open('gpurun_out/sched_$name.json'))['value'])"
done
