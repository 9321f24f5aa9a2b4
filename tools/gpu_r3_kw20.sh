#!/bin/bash
# Round 3: radix-2^20 key combs.  The committee / certificate GPU tests, then
# C3 and C1 through bench.py with the radix-2^20 key combs (default) and the
# radix-2^16 ones (COA_KEY_WCOMB20_MB=0), alternated.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_committee.py tests/test_gpu_c3.py tests/test_gpu_certificates.py tests/test_gpu_queue_harness.py tests/test_queue.py -m gpu > gpurun_out/kw20_tests.log 2>&1 \
  || { tail -30 gpurun_out/kw20_tests.log; exit 1; }
tail -2 gpurun_out/kw20_tests.log
for rep in 1 2; do
  for mb in default 0; do
    if [ "$mb" = default ]; then unset COA_KEY_WCOMB20_MB; else export COA_KEY_WCOMB20_MB=$mb; fi
    timeout -k 10 300 python3 bench.py --steps 5 --no-cpu-baseline --sections c3_certificate_verify,c1_certificate_verify \
      > gpurun_out/kw20_$mb.json 2> gpurun_out/kw20_$mb.err || { tail -20 gpurun_out/kw20_$mb.err; exit 1; }
    python3 -c "
import json; s=json.load(open('gpurun_out/kw20_$mb.json'))['secondary']
c3=s['c3_certificate_verify']; c1=s['c1_certificate_verify']
print('key wcomb20 MB=$mb', 'C3', round(c3['certs_per_s']/1e6,3), 'M/s reg', c3['register_ms'], 'ms p50', c3['c_caller']['p50_ms'], '| C1', round(c1['certs_per_s']/1e6,3), 'M/s p50', c1['c_caller']['p50_ms'])"
  done
done
