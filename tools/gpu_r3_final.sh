#!/bin/bash
# Round 3 record on the final tree: the driver's bench command, then the same
# command under the kernel trace (per-kernel stats by grid for profiles/).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
SECONDS=0; timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err \
  || { tail -20 gpurun_out/final_bench.err; exit 1; }
echo "bench wall ${SECONDS} s"
python3 -c "import json; d=json.load(open('gpurun_out/final_bench.json')); print({k: d[k] for k in ('value','ms_per_step')}, d['roofline']['frac'], [k for k,v in d['secondary'].items() if 'error' in v])"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/final_prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final_prof_bench.json 2> gpurun_out/final_prof.err \
  || { tail -20 gpurun_out/final_prof.err; exit 1; }
python3 tools/kernel_trace_summary.py gpurun_out/final_prof gpurun_out/final_by_grid.json | head -30
