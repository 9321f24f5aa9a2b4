#!/bin/bash
# Same-box A/B of one environment switch VAR over the values KINDS on
# bench.py's host_e2e section (host-pointer C2 from 1/2/4 C threads over as
# many contexts, host C3), REPS alternations, one process each.  Round 5
# used it for COA_CTX_STREAMS and COA_HOST_PIN (both since removed;
# profiles/r05_host_c2_threads_ab.txt).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
for rep in $(seq ${REPS:-3}); do
  for kind in ${KINDS:?}; do
    env ${VAR:?}=$kind timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 2 --sections host_e2e \
      > gpurun_out/he_$kind.json 2> gpurun_out/he_$kind.err || exit 1
    python -c "import json;s=json.load(open('gpurun_out/he_$kind.json'))['summary'];print('$kind', $rep, s['host_c2_verify_per_s'], s['host_c3_certs_per_s'], s['c3_stream_certs_per_s'])"
  done
done
