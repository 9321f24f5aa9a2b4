# GPU session (round 5): queue tests, then an A/B of direct launches by
# submitting threads (COA_QUEUE_DIRECT) on the round mixes; every step under
# its own time limit.
set -o pipefail
mkdir -p gpurun_out/dir
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_queue.py tests/test_gpu_queue_harness.py tests/test_gpu_recovery.py > gpurun_out/dir/tests.log 2>&1 || exit 1
for r in 1 2; do
  for v in 1 0; do
    COA_QUEUE_DIRECT=$v timeout -k 10 240 python bench.py --no-cpu-baseline --sections queue_round_mix,queue_round_mix_c1 > gpurun_out/dir/mix_${v}_$r.json 2> gpurun_out/dir/mix_${v}_$r.err || exit 1
  done
done
