#!/bin/bash
# Round 3, row products: the A/B microbenchmark, the whole GPU suite, then the
# latency sections of the bench (single verify, verify_batch, C1) on this build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 60 ./tools/ubench_rows3 > gpurun_out/ubench_rows3.txt 2>&1 || { cat gpurun_out/ubench_rows3.txt; exit 1; }
cat gpurun_out/ubench_rows3.txt
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
  || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py --steps 20 --no-cpu-baseline --sections verify_single,verify_batch,c1_certificate_verify \
  > gpurun_out/bench_lat.json 2> gpurun_out/bench_lat.err || { tail -20 gpurun_out/bench_lat.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_lat.json')); s=d['secondary']
print('C2', d['value']); print(json.dumps(s['verify_single'])); print(json.dumps(s['verify_batch']['single_group'])); c=s['c1_certificate_verify']; print('C1 p50', c['p50_ms'], c['c_caller'])"
