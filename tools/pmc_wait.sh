#!/bin/bash
# SQ issue/wait shares of the C2 verify call (one counter pass):
# profiles/r02_verify_pmc_wait.json via tools/pmc_wait_summary.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 5 -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
  SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INSTS_BRANCH -T -d gpurun_out/pmc_any -o run --output-format csv \
  -- python3 bench.py --no-cpu-baseline --no-secondary --steps 3 --warmup 1 > gpurun_out/pmc_any.json 2> gpurun_out/pmc_any.err
