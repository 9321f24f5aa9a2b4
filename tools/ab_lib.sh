#!/bin/bash
# Same-box A/B of engine builds on the C2 bench line: LIBS="name=path ..."
# (default: the in-tree library against build/ab/libcoa_verify_base.so),
# alternating REPS times; N triples per call (default C2).  One line per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
LIBS=${LIBS:-"new=xrpl-coa-prototype_amd/lib/libcoa_verify.so base=build/ab/libcoa_verify_base.so"}
for rep in $(seq ${REPS:-3}); do
  for kv in $LIBS; do
    name=${kv%%=*}; lib=${kv#*=}
    COA_VERIFY_LIB=$PWD/$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-secondary --steps 40 --n ${N:-65536} \
      > gpurun_out/ab_$name.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ab_$name.json'));print('$name', d['value'], d['kernel_ms'], d['verdicts_ok'])"
  done
done
