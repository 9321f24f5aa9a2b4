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
if [[ $STEPS == *pmc* ]]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    run "pmc $c" && timeout -k 10 300 rocprofv3 --pmc $c -T -d gpurun_out/pmc_$c -o run --output-format csv \
        -- python3 bench.py --no-cpu-baseline --no-secondary --steps 3 --warmup 1 > gpurun_out/pmc_$c.json 2> gpurun_out/pmc_$c.err \
      || { tail -30 gpurun_out/pmc_$c.err; exit 1; }
  done
  find gpurun_out -path "*pmc_*" -name "*.csv" | head
fi
