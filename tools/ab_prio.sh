#!/bin/bash
# A/B of the k_pre_halve hash-role wave priority (COA_PRE_PRIO), alternating,
# C2 size and a C5 shard; one JSON summary line per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
for cfg in "1 65536" "0 65536" "1 65536" "0 65536" "1 2097152" "0 2097152"; do
  set -- $cfg
  COA_PRE_PRIO=$1 timeout -k 10 120 python bench.py --no-cpu-baseline --no-secondary --steps 40 --n $2 > gpurun_out/ab_prio_$1_$2.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab_prio_$1_$2.json'));print('prio $1 n $2', d['value'], d['kernel_ms'], d['verdicts_ok'])"
done
