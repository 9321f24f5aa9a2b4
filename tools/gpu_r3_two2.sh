#!/bin/bash
# Round 3: k_verify_main2 threshold at a quarter wave per SIMD of items.
# Verify parity tests, A/B around the threshold, the C2 counters on these
# sources (copied into this box's profiles/ so the bench line ties them),
# then the final bench line and its kernel trace (tools/gpu_r3_final.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_adversarial.py tests/test_gpu_verify.py tests/test_queue.py -m gpu > gpurun_out/two2_tests.log 2>&1 \
  || { tail -30 gpurun_out/two2_tests.log; exit 1; }
tail -2 gpurun_out/two2_tests.log
for n in 16384 24576; do
  echo "n=$n"; ENVS="one=COA_MAIN_TWO=0 default" REPS=1 N=$n bash tools/ab_env.sh || exit 1
done
bash tools/gpu_round.sh verifypmc || exit 1
cp gpurun_out/verify_pmc.json profiles/r03_verify_pmc.json || exit 1
bash tools/pmc_wait.sh || exit 1
bash tools/gpu_r3_final.sh
