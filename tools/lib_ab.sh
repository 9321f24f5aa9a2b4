#!/bin/bash
# Same-box A/B of engine builds on one bench section: LIBS="name=path ..."
# (path = a libcoa_verify.so with its liblatc.so beside it, e.g. build/r5/
# from an older commit; "default" = the tree's own lib), SECTION (default
# host_e2e), REPS alternations, one process each; prints each run's summary
# keys KEYS (default the C3 stream and host lines).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
SECTION=${SECTION:-host_e2e}
KEYS=${KEYS:-host_c3_certs_per_s c3_stream_certs_per_s c3_stream_copied_certs_per_s c3_stream_paced_4_producers}
for rep in $(seq ${REPS:-3}); do
  for lv in ${LIBS:?}; do
    name=${lv%%=*}
    path=${lv#*=}
    out=gpurun_out/lab_${name}_$rep
    if [ "$path" = default ]; then
      timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 2 --sections $SECTION \
        --secondary-out $out.sec.json > $out.json 2> $out.err || exit 1
    else
      COA_VERIFY_LIB=$path timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 2 \
        --sections $SECTION --secondary-out $out.sec.json > $out.json 2> $out.err || exit 1
    fi
    python -c "import json,sys;s=json.loads(open('$out.json').read().strip().splitlines()[-1])['summary'];print('$name', $rep, *[(k, s.get(k)) for k in sys.argv[1:]])" $KEYS
  done
done
