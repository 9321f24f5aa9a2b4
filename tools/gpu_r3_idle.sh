#!/bin/bash
# Round 3: the queue's idle-launch window policy.  Queue GPU tests, then the
# committee-100 round mix under both policies (bench.py queue_round_mix).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_queue.py tests/test_gpu_queue_harness.py -m gpu > gpurun_out/idle_tests.log 2>&1 \
  || { tail -30 gpurun_out/idle_tests.log; exit 1; }
tail -2 gpurun_out/idle_tests.log
timeout -k 10 300 python3 bench.py --steps 5 --no-cpu-baseline --sections queue_round_mix > gpurun_out/idle_mix.json 2> gpurun_out/idle_mix.err \
  || { tail -20 gpurun_out/idle_mix.err; exit 1; }
python3 -c "
import json; s=json.load(open('gpurun_out/idle_mix.json'))['secondary']['queue_round_mix']
for key in ('rates', 'rates_idle_launch'):
    for r, row in s[key].items():
        print(key, r, 'windows', row['windows'], 'req/win', row['mean_requests_per_window'], 'cert p50/p99', row['certificate']['p50_ms'], row['certificate']['p99_ms'], 'sig p50/p99', row['signature']['p50_ms'], row['signature']['p99_ms'])"
