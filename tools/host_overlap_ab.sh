# GPU session (round 5): host-pointer verify tests, then host_e2e with and
# without the two-stream halves (COA_HOST_OVERLAP), alternating.
set -o pipefail
mkdir -p gpurun_out/ho
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_adversarial.py tests/test_gpu_verify.py tests/test_gpu_c5.py tests/test_gpu_recovery.py > gpurun_out/ho/tests.log 2>&1 || exit 1
for r in 1 2; do
  for v in 1 0; do
    COA_HOST_OVERLAP=$v timeout -k 10 300 python bench.py --no-cpu-baseline --sections host_e2e > gpurun_out/ho/he_${v}_$r.json 2> gpurun_out/ho/he_${v}_$r.err || exit 1
  done
done
