#!/bin/bash
# Round 3: one-certificate latency calls read in place from coherent
# page-locked memory (default) vs staged through an H2D copy
# (COA_CERT_ZEROCOPY=0).  Certificate GPU tests, then C3 / C1 p50 alternated.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_committee.py tests/test_gpu_certificates.py tests/test_gpu_c3.py -m gpu > gpurun_out/zc_tests.log 2>&1 \
  || { tail -30 gpurun_out/zc_tests.log; exit 1; }
tail -2 gpurun_out/zc_tests.log
for rep in 1 2; do
  for zc in 1 0; do
    export COA_CERT_ZEROCOPY=$zc
    timeout -k 10 300 python3 bench.py --steps 5 --no-cpu-baseline --sections c3_certificate_verify,c1_certificate_verify \
      > gpurun_out/zc_$zc.json 2> gpurun_out/zc_$zc.err || { tail -20 gpurun_out/zc_$zc.err; exit 1; }
    python3 -c "
import json; s=json.load(open('gpurun_out/zc_$zc.json'))['secondary']
c3=s['c3_certificate_verify']; c1=s['c1_certificate_verify']
print('zerocopy=$zc', 'C3 p50', c3['p50_ms'], 'C caller', c3['c_caller']['p50_ms'], c3['c_caller']['p99_ms'], '| C1 p50', c1['p50_ms'], 'C caller', c1['c_caller']['p50_ms'])"
  done
done
