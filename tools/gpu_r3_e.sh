#!/bin/bash
# round 3: Lehmer halving -- parity, same-box A/B against the previous build,
# the [e]B-placement A/B, single-verify latency, and the streamed C4 with
# more hardware queues
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_halve.py tests/test_gpu_adversarial.py tests/test_gpu_latency.py tests/test_gpu_verify.py -x -q --timeout 240 --timeout-method thread > gpurun_out/t_halve.log 2>&1 || { tail -30 gpurun_out/t_halve.log; exit 1; }
tail -2 gpurun_out/t_halve.log
REPS=3 bash tools/ab_lib.sh || exit 1
for r in 1 2; do for eb in 0 1; do
  COA_SPLIT_EB=$eb timeout -k 10 120 python bench.py --steps 40 --no-cpu-baseline --no-secondary > gpurun_out/ab_eb${eb}_r$r.json 2>> gpurun_out/ab.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ab_eb${eb}_r$r.json'));print('eb=$eb', d['value'], d['kernel_ms'], d['verdicts_ok'])"
done; done
timeout -k 10 200 python bench.py --steps 3 --sections verify_single > gpurun_out/vs.json 2>> gpurun_out/ab.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/vs.json'))['secondary']['verify_single'];print({k:(v['p50_ms'],v['c_caller']['p50_ms']) for k,v in d.items() if isinstance(v,dict)}, d['cpu_single_thread_p50_ms'])"
for hq in 8; do
  GPU_MAX_HW_QUEUES=$hq COA_QUEUE_SLOTS=4 timeout -k 10 200 python bench.py --steps 3 --no-cpu-baseline --sections c4_stream > gpurun_out/c4_hq$hq.json 2>> gpurun_out/ab.err || exit 1
  python3 -c "
import json;c=json.load(open('gpurun_out/c4_hq$hq.json'))['secondary']['c4_stream']; print('hwq $hq', {k:(v['p50_ms'],v['p99_ms'],v['achieved_batches_per_s'],v['windows']) for k,v in c.items() if k.startswith('rate')})"
done
