cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_queue_harness.py tests/test_gpu_recovery.py tests/test_queue.py -x -v --timeout 240 --timeout-method thread > gpurun_out/t1.log 2>&1 || { tail -40 gpurun_out/t1.log; exit 1; }
tail -15 gpurun_out/t1.log
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
for p in 1 2 4 8 16; do COA_QUEUE_SLOTS=2 timeout -k 10 120 ./tools/queue_probe 4194304 $p 65536 200 1 >> gpurun_out/queue_probe.jsonl 2>> gpurun_out/queue_probe.err || exit 1; tail -1 gpurun_out/queue_probe.jsonl; done
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
