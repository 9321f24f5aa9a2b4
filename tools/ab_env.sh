#!/bin/bash
# Same-box A/B of a runtime switch on the C2 bench line: ENVS="name=VAR=value ..."
# (a name with no assignment runs the default), alternating REPS times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
ENVS=${ENVS:-"ebmain=COA_SPLIT_EB=0 default"}
for rep in $(seq ${REPS:-3}); do
  for kv in $ENVS; do
    name=${kv%%=*}; assign=${kv#*=}; [ "$assign" = "$kv" ] && assign=""
    env $assign timeout -k 10 120 python bench.py --no-cpu-baseline --no-secondary --steps 40 --n ${N:-65536} \
      > gpurun_out/abe_$name.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/abe_$name.json'));print('$name', d['value'], d['kernel_ms'], d['verdicts_ok'])"
  done
done
