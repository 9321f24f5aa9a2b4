#!/bin/bash
# Round 3: k_verify_main's prologue loads issued together.  Verify GPU tests,
# then C2 alternating the new library and the previous one (lib/ab/).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_adversarial.py tests/test_gpu_verify.py tests/test_gpu_c5.py -m gpu > gpurun_out/pro_tests.log 2>&1 \
  || { tail -30 gpurun_out/pro_tests.log; exit 1; }
tail -2 gpurun_out/pro_tests.log
for rep in 1 2 3; do
  for lib in new prev; do
    if [ "$lib" = new ]; then unset COA_VERIFY_LIB; else export COA_VERIFY_LIB=$PWD/xrpl-coa-prototype_amd/lib/ab/libcoa_verify_prev.so; fi
    timeout -k 10 200 python3 bench.py --steps 200 --no-cpu-baseline --no-secondary > gpurun_out/pro_$lib.json 2> gpurun_out/pro_$lib.err || { tail -20 gpurun_out/pro_$lib.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/pro_$lib.json')); print('$lib', round(d['value']/1e6,2), d['ms_per_step'])"
  done
done
