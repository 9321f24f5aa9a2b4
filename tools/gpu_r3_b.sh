#!/bin/bash
# round 3: new bench sections (streamed C4, paced committee-100 round mix) and
# the callback-helper A/B of the aggregation queue
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -X faulthandler bench.py --steps 5 --no-cpu-baseline --sections c4_sha512,c4_stream,queue_round_mix > gpurun_out/bench_sec.json 2> gpurun_out/bench_sec.err || { tail -30 gpurun_out/bench_sec.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_sec.json'));print(json.dumps(d['secondary'],indent=1))"
for h in 0 3; do for p in 4 8 16; do COA_QUEUE_HELPERS=$h timeout -k 10 120 ./tools/queue_probe 4194304 $p 65536 200 1 > gpurun_out/qp_h${h}_p${p}.json 2>> gpurun_out/queue_probe.err || exit 1; echo "helpers=$h $(cat gpurun_out/qp_h${h}_p${p}.json | cut -c1-400)"; done; done
