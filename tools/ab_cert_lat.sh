#!/bin/bash
# Same-box A/B of the certificate latency (C1/C3 p50) between the in-tree
# library and LIB_B (default build/ab/libcoa_verify_prev.so): the certificate
# GPU tests first, then alternating secondary-only bench runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 5 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_committee.py \
  tests/test_gpu_certificates.py tests/test_gpu_c3.py > gpurun_out/t_cert.log 2>&1; tail -2 gpurun_out/t_cert.log
grep -q passed gpurun_out/t_cert.log && ! grep -q failed gpurun_out/t_cert.log || exit 1
LIB_B=${LIB_B:-build/ab/libcoa_verify_prev.so}
for rep in $(seq ${REPS:-2}); do
  for kv in new=xrpl-coa-prototype_amd/lib/libcoa_verify.so old=$LIB_B; do
    name=${kv%%=*}; lib=${kv#*=}
    COA_VERIFY_LIB=$PWD/$lib timeout -k 10 240 python bench.py --no-cpu-baseline --steps 5 --warmup 1 --c4-batches "" \
      > gpurun_out/abc_$name.json 2>gpurun_out/abc_$name.err || { tail -5 gpurun_out/abc_$name.err; exit 1; }
    python -c "
import json;d=json.load(open('gpurun_out/abc_$name.json'))['secondary']
c3=d['c3_certificate_verify'];c1=d['c1_certificate_verify']
def p(x): return {k:v for k,v in x.items() if 'p50' in k or k in ('certs_per_s','c_caller')}
print('$name C3', p(c3)); print('$name C1', p(c1))"
  done
done
