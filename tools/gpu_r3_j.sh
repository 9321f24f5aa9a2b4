#!/bin/bash
# verify_batch latency prefilter: parity (batch, msm, committee), then the
# one-group p50 both routes, then a kernel trace of the prefilter route
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_msm.py tests/test_gpu_latency.py > gpurun_out/j_tests.log 2>&1 || { tail -30 gpurun_out/j_tests.log; exit 1; }
tail -2 gpurun_out/j_tests.log
timeout -k 10 120 python3 tools/msm1_probe.py 67 300 || exit 1
COA_BATCH_LAT=0 timeout -k 10 120 python3 tools/msm1_probe.py 67 300 || exit 1
timeout -k 10 120 python3 tools/msm1_probe.py 3 300 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/msm1p -o run --output-format csv -- python3 tools/msm1_probe.py 67 50 > gpurun_out/msm1p.json 2> gpurun_out/msm1p.err || { tail -20 gpurun_out/msm1p.err; exit 1; }
COA_BATCH_LAT=0 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/msm1x -o run --output-format csv -- python3 tools/msm1_probe.py 67 50 > gpurun_out/msm1x.json 2> gpurun_out/msm1x.err || { tail -20 gpurun_out/msm1x.err; exit 1; }
