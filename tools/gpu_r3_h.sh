#!/bin/bash
# round 3: certificate digests once per certificate (prologue kernel) and the
# 3-wave certificate kernel: parity, then C3 / C1 A/B
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_committee.py tests/test_gpu_c3.py tests/test_gpu_certificates.py tests/test_queue.py -x -q --timeout 240 --timeout-method thread > gpurun_out/t_cert.log 2>&1 || { tail -30 gpurun_out/t_cert.log; exit 1; }
tail -1 gpurun_out/t_cert.log
COA_CERT_WAVES=3 timeout -k 10 500 python -u -m pytest tests/test_gpu_c3.py -x -q --timeout 240 --timeout-method thread > gpurun_out/t_cert3.log 2>&1 || { tail -30 gpurun_out/t_cert3.log; exit 1; }
tail -1 gpurun_out/t_cert3.log
for r in 1 2; do for v in "base=COA_CERT_DIGEST_PER_VOTE=1" "dig=X=1" "w3=COA_CERT_WAVES=3"; do
name=${v%%=*}; ev=${v#*=}
env $ev timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --sections c3_certificate_verify,c1_certificate_verify --cpu-thread-seconds 1 > gpurun_out/c3_$name.json 2>> gpurun_out/ab.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/c3_$name.json'))['secondary'];print('$name', {k:(v['certs_per_s'],v['round_ms'],v['c_caller']['p50_ms']) for k,v in d.items()})"
done; done
