#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; steps are chained with && so the
# first failure ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS="${1:-tests,smoke,bench,prof}"
run() { echo "== $1" ; }
if [[ $STEPS == *tests* ]]; then
  run tests && timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
    || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
fi
if [[ $STEPS == *smoke* ]]; then
  run smoke && timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
    || { tail -30 gpurun_out/smoke.log; exit 1; }
  tail -2 gpurun_out/smoke.log
fi
if [[ $STEPS == *bench* ]]; then
  run bench && timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err \
    || { tail -30 gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
if [[ $STEPS == *big* ]]; then
  run bench_big && timeout -k 10 300 python bench.py --n 524288 --steps 10 --no-cpu-baseline --no-secondary > gpurun_out/bench_big.json 2> gpurun_out/bench_big.err \
    || { tail -30 gpurun_out/bench_big.err; exit 1; }
  cat gpurun_out/bench_big.json
fi
if [[ $STEPS == *prof* ]]; then
  run prof && timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof -o run --output-format csv \
      -- python3 bench.py --no-cpu-baseline --no-secondary --steps 10 > gpurun_out/bench_prof.json 2> gpurun_out/prof.err \
    || { tail -30 gpurun_out/prof.err; exit 1; }
  find gpurun_out/prof -name "*stats*" | head
  for f in $(find gpurun_out/prof -name "*kernel_stats.csv"); do cat "$f"; done
fi
if [[ $STEPS == *sq* ]]; then
  run "pmc SQ" && timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -T -d gpurun_out/pmc_SQ -o run --output-format csv \
      -- python3 bench.py --no-cpu-baseline --no-secondary --steps 3 --warmup 1 > gpurun_out/pmc_SQ.json 2> gpurun_out/pmc_SQ.err \
    || { tail -30 gpurun_out/pmc_SQ.err; exit 1; }
fi
if [[ $STEPS == *fullprof* ]]; then
  # the driver's exact command (python bench.py, defaults) under the kernel trace
  run fullprof && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/fullprof -o run --output-format csv \
      -- python3 bench.py > gpurun_out/bench_fullprof.json 2> gpurun_out/fullprof.err \
    || { tail -30 gpurun_out/fullprof.err; exit 1; }
  python3 tools/kernel_trace_summary.py gpurun_out/fullprof gpurun_out/fullprof_by_grid.json > gpurun_out/fullprof_summary.txt
fi
if [[ $STEPS == *verifypmc* ]]; then
  # three counter passes of the C2 verify call -> profiles JSON tied to this build
  run "pmc SQ" && timeout -k 10 -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -T -d gpurun_out/vp/pmc_SQ -o run --output-format csv \
      -- python3 bench.py --no-cpu-baseline --no-secondary --steps 3 --warmup 1 > gpurun_out/vp_sq.json 2> gpurun_out/vp_sq.err \
    || { tail -30 gpurun_out/vp_sq.err; exit 1; }
  for c in FETCH_SIZE WRITE_SIZE; do
    run "pmc $c" && timeout -k 10 -s KILL 240 rocprofv3 --pmc $c -T -d gpurun_out/vp/pmc_$c -o run --output-format csv \
        -- python3 bench.py --no-cpu-baseline --no-secondary --steps 3 --warmup 1 > gpurun_out/vp_$c.json 2> gpurun_out/vp_$c.err \
      || { tail -30 gpurun_out/vp_$c.err; exit 1; }
  done
  python3 tools/pmc_verify.py gpurun_out/vp 65536 gpurun_out/verify_pmc.json > /dev/null && echo "verify_pmc ok"
fi
if [[ $STEPS == *pmc* ]] && [[ $STEPS != *verifypmc* ]]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    run "pmc $c" && timeout -k 10 300 rocprofv3 --pmc $c -T -d gpurun_out/pmc_$c -o run --output-format csv \
        -- python3 bench.py --no-cpu-baseline --no-secondary --steps 3 --warmup 1 > gpurun_out/pmc_$c.json 2> gpurun_out/pmc_$c.err \
      || { tail -30 gpurun_out/pmc_$c.err; exit 1; }
  done
  find gpurun_out -path "*pmc_*" -name "*.csv" | head
fi
if [[ $STEPS == *latprobe* ]]; then
  run latprobe && timeout -k 10 300 python3 tools/lat_probe.py > gpurun_out/lat_probe.jsonl 2> gpurun_out/lat_probe.err \
    || { tail -30 gpurun_out/lat_probe.err; exit 1; }
  cat gpurun_out/lat_probe.jsonl
fi
if [[ $STEPS == *onlytests* ]]; then
  run onlytests && timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread $TESTS > gpurun_out/pytest_sel.log 2>&1 \
    || { tail -40 gpurun_out/pytest_sel.log; exit 1; }
  tail -15 gpurun_out/pytest_sel.log
fi
if [[ $STEPS == *vlat* ]]; then
  run vlat && timeout -k 10 120 python3 tools/vlat_trace.py run > gpurun_out/vlat_trace.jsonl 2> gpurun_out/vlat_trace.err \
    || { tail -30 gpurun_out/vlat_trace.err; exit 1; }
  cat gpurun_out/vlat_trace.jsonl
fi
