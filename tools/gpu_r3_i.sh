#!/bin/bash
# round 3: C2 with 4 vs 8 HIP hardware queues (A/B), queue tests with four
# slots, and the 2-rank torchrun path with both ranks on this box's GPU
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_queue.py tests/test_gpu_queue_harness.py -x -q --timeout 240 --timeout-method thread > gpurun_out/t_q.log 2>&1 || { tail -30 gpurun_out/t_q.log; exit 1; }
tail -1 gpurun_out/t_q.log
for r in 1 2 3; do for hq in 4 8; do
  GPU_MAX_HW_QUEUES=$hq timeout -k 10 120 python bench.py --steps 40 --no-cpu-baseline --no-secondary > gpurun_out/ab_hq${hq}_r$r.json 2>> gpurun_out/ab.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ab_hq${hq}_r$r.json'));print('hwq=$hq', d['value'], d['kernel_ms'], d['verdicts_ok'])"
done; done
COA_BENCH_ONE_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 > gpurun_out/bench_2rank.json 2> gpurun_out/bench_2rank.err || { tail -20 gpurun_out/bench_2rank.err; exit 1; }
cat gpurun_out/bench_2rank.json | cut -c1-400
# k_pre_halve role timing on this build (diagnostic library: build/diag)
for diag in 0 4 2; do
  COA_VERIFY_LIB=$PWD/build/diag/libcoa_verify.so COA_PRE_DIAG=$diag timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/roles_$diag -o run --output-format csv \
    -- python3 tools/inflight_probe.py 65536 20 > gpurun_out/roles_$diag.jsonl 2>&1 || exit 1
  f=$(find gpurun_out/roles_$diag -name "*kernel_stats.csv" | head -1)
  echo "diag $diag: $(grep -h 'k_pre_halve' $f | cut -d, -f1-4 | cut -c1-40,200-400)"
done
