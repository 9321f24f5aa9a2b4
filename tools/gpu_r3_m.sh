#!/bin/bash
# prefilter with the [2^252]A doubling chain on wave 2: parity, then p50
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_latency.py tests/test_gpu_committee.py > gpurun_out/m_tests.log 2>&1 || { tail -30 gpurun_out/m_tests.log; exit 1; }
tail -2 gpurun_out/m_tests.log
timeout -k 10 120 python3 tools/msm1_probe.py 67 300 || exit 1
timeout -k 10 120 python3 tools/msm1_probe.py 3 300 || exit 1
COA_BATCH_LAT=0 timeout -k 10 120 python3 tools/msm1_probe.py 67 300 || exit 1
timeout -k 10 120 python3 tools/msm1_probe.py 3 200 300 || exit 1
COA_BATCH_LAT=0 timeout -k 10 120 python3 tools/msm1_probe.py 3 200 300 || exit 1
