#!/bin/bash
# round 3 A/B: [e]B in k_pre_halve's hash role (COA_SPLIT_EB=1) against
# k_verify_main (default), alternated; then the streamed C4 with more HIP
# hardware queues (GPU_MAX_HW_QUEUES) and queue slots
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out
for r in 1 2 3; do for eb in 0 1; do
  COA_SPLIT_EB=$eb timeout -k 10 120 python bench.py --steps 40 --no-cpu-baseline --no-secondary > gpurun_out/ab_eb${eb}_r$r.json 2>> gpurun_out/ab.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ab_eb${eb}_r$r.json'));print('eb=$eb', d['value'], d['kernel_ms'], d['verdicts_ok'])"
done; done
for hq in 4 8; do
  GPU_MAX_HW_QUEUES=$hq COA_QUEUE_SLOTS=4 timeout -k 10 200 python bench.py --steps 3 --no-cpu-baseline --sections c4_stream > gpurun_out/c4_hq$hq.json 2>> gpurun_out/ab.err || exit 1
  python3 -c "
import json;c=json.load(open('gpurun_out/c4_hq$hq.json'))['secondary']['c4_stream']; print('hwq $hq', {k:(v['p50_ms'],v['p99_ms'],v['achieved_batches_per_s'],v['windows']) for k,v in c.items() if k.startswith('rate')})"
done
