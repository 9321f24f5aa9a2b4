#!/bin/bash
# Round 3: k_verify_main2 (an item's two chains in two waves; default below
# half a wave per SIMD of items).  The whole GPU suite and smoke on the
# default switch, same-box A/B against the one-wave main kernel at 4k / 16k /
# 32k items and C2, then the C2 counters on these sources (sha-tied).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/two_tests.log 2>&1 \
  || { tail -30 gpurun_out/two_tests.log; exit 1; }
tail -2 gpurun_out/two_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
for n in 4096 16384 32768 65536; do
  echo "n=$n"; ENVS="one=COA_MAIN_TWO=0 default" REPS=2 N=$n bash tools/ab_env.sh || exit 1
done
bash tools/gpu_round.sh verifypmc || exit 1
bash tools/pmc_wait.sh
