#!/bin/bash
# Round-end GPU session: the GPU test suite, smoke(), the driver's bench
# command, and a kernel trace (--kernel-trace --stats) of the same command.
# Every GPU step has its own time limit; the first failure ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
T=${TAG:-final}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 \
  || { tail -30 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --secondary-out gpurun_out/${T}_bench_secondary.json \
  > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -30 gpurun_out/${T}_bench.err; exit 1; }
tail -c 600 gpurun_out/${T}_bench.json
rm -rf gpurun_out/${T}_prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv \
  -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --secondary-out gpurun_out/${T}_prof_secondary.json \
  > gpurun_out/${T}_prof_bench.json 2> gpurun_out/${T}_prof.err || { tail -30 gpurun_out/${T}_prof.err; exit 1; }
python3 tools/kernel_trace_summary.py gpurun_out/${T}_prof gpurun_out/${T}_prof_by_grid.json > gpurun_out/${T}_prof_summary.txt \
  || exit 1
find gpurun_out/${T}_prof -name "*kernel_stats.csv" -exec head -6 {} \;
# the trace itself is large: keep the summaries only
find gpurun_out/${T}_prof -name "*kernel_trace.csv" -delete
