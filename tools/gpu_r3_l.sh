#!/bin/bash
# C2 with calls in flight (bench secondary), then the one-group Pippenger run sweep
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python3 -X faulthandler bench.py --no-cpu-baseline --sections c2_inflight --steps 20 --warmup 3 > gpurun_out/l_bench.json 2> gpurun_out/l_bench.err || { tail -20 gpurun_out/l_bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/l_bench.json').read().splitlines()[-1]);print(d['value'], json.dumps(d['secondary']['c2_inflight']))"
bash tools/gpu_r3_k.sh
