#!/bin/bash
# round 3: queue parity after the latency-kernel route for small windows,
# then the paced sections at 2 / 4 / 8 slots per GPU
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_queue_harness.py tests/test_queue.py tests/test_gpu_recovery.py -x -q --timeout 240 --timeout-method thread > gpurun_out/t_queue.log 2>&1 || { tail -30 gpurun_out/t_queue.log; exit 1; }
tail -2 gpurun_out/t_queue.log
for sl in 2 4 8; do
  COA_QUEUE_SLOTS=$sl timeout -k 10 300 python -X faulthandler bench.py --steps 3 --no-cpu-baseline --sections c4_stream,queue_round_mix > gpurun_out/bench_sec_s$sl.json 2> gpurun_out/bench_sec_s$sl.err || { tail -30 gpurun_out/bench_sec_s$sl.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/bench_sec_s$sl.json'))['secondary']
c=d['c4_stream']; print('slots $sl c4', {k:(v['p50_ms'],v['p99_ms'],v['achieved_batches_per_s'],v['windows']) for k,v in c.items() if k.startswith('rate')})
q=d['queue_round_mix']['rates']; print('slots $sl mix', {k:(v['certificate']['p50_ms'],v['certificate']['p99_ms'],v['signature']['p50_ms'],v['signature']['p99_ms'],v['windows']) for k,v in q.items()})"
done
