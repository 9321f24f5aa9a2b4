#!/bin/bash
# Same-box A/B of one environment switch on bench sections: VAR, KINDS
# ("v1 v2 ..."), SECTION (comma list, default host_e2e), REPS alternations,
# one process each; prints each run's summary keys KEYS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
SECTION=${SECTION:-host_e2e}
KEYS=${KEYS:-host_c3_certs_per_s c3_stream_certs_per_s c3_stream_paced_4_producers}
for rep in $(seq ${REPS:-3}); do
  for kind in ${KINDS:?}; do
    out=gpurun_out/eab_${kind}_$rep
    env ${VAR:?}=$kind timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 2 \
      --sections $SECTION --secondary-out $out.sec.json > $out.json 2> $out.err || exit 1
    python -c "import json,sys;s=json.loads(open('$out.json').read().strip().splitlines()[-1])['summary'];print('$kind', $rep, *[(k, s.get(k)) for k in sys.argv[1:]])" $KEYS
  done
done
