#!/bin/bash
# Round 3: B's wide comb in radix 2^24 (11 positions, 8.9 GB) against radix
# 2^20 (13 positions, 654 MB; the previous build, lib/ab/).  Self-test of the
# whole table and the verify / certificate GPU tests on the new build, then
# C2 + C3 + C1 through bench.py alternating the two libraries.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_committee.py tests/test_gpu_c3.py tests/test_gpu_certificates.py tests/test_gpu_adversarial.py tests/test_gpu_verify.py tests/test_gpu_latency.py tests/test_gpu_batch.py -m gpu > gpurun_out/bw24_tests.log 2>&1 \
  || { tail -30 gpurun_out/bw24_tests.log; exit 1; }
tail -2 gpurun_out/bw24_tests.log
for rep in 1 2; do
  for lib in new w20; do
    if [ "$lib" = new ]; then unset COA_VERIFY_LIB; else export COA_VERIFY_LIB=$PWD/xrpl-coa-prototype_amd/lib/ab/libcoa_verify_w20.so; fi
    timeout -k 10 300 python3 bench.py --steps 40 --no-cpu-baseline --sections c3_certificate_verify,c1_certificate_verify \
      > gpurun_out/bw24_$lib.json 2> gpurun_out/bw24_$lib.err || { tail -20 gpurun_out/bw24_$lib.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/bw24_$lib.json')); s=d['secondary']
c3=s['c3_certificate_verify']; c1=s['c1_certificate_verify']
print('$lib', 'C2', round(d['value']/1e6,2), '| C3', round(c3['certs_per_s']/1e6,3), 'M/s p50', c3['c_caller']['p50_ms'], '| C1', round(c1['certs_per_s']/1e6,3), 'M/s p50', c1['c_caller']['p50_ms'])"
  done
done
