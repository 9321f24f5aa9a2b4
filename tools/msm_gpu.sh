export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_msm.py -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_msm.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_msm.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/msm_probe.py 65536 262144 524288 2097152 > gpurun_out/msm_probe.log 2>&1 || exit 1
cat gpurun_out/msm_probe.log
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_msm3 -o msm -- python3 $GRAFT_REPO_ROOT/tools/msm_probe.py 65536 2097152 > $GRAFT_REPO_ROOT/gpurun_out/prof_msm3.log 2>&1; echo prc=$?
