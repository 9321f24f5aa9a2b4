#!/bin/bash
# headline timing A/B: settle phase and step counts (alternating, same box)
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out
for rep in 1 2; do
  for v in "--settle-s 0 --steps 20 --warmup 3" "--settle-s 0 --steps 100 --warmup 10" "--settle-s 0.3 --steps 100 --warmup 10" "--settle-s 0.3 --steps 20 --warmup 3"; do
    out=$(timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-secondary $v) || exit 1
    echo "$v :: $(echo "$out" | tail -1 | python3 -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"], d["ms_per_step"])')"
  done
done
