#!/bin/bash
# round 3: certificate kernel with dynamic chunk grabbing (parity + C3/C1),
# k_pre_halve priority for the [e]B additions (A/B), then the kernel trace of
# the C2 bench on this build
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_committee.py tests/test_gpu_c3.py tests/test_gpu_certificates.py tests/test_queue.py tests/test_gpu_adversarial.py -x -q --timeout 240 --timeout-method thread > gpurun_out/t_cert.log 2>&1 || { tail -30 gpurun_out/t_cert.log; exit 1; }
tail -1 gpurun_out/t_cert.log
timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --sections c3_certificate_verify,c1_certificate_verify --cpu-thread-seconds 2 > gpurun_out/c3.json 2>> gpurun_out/ab.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/c3.json'))['secondary'];print({k:(v['certs_per_s'],v['round_ms'],v['c_caller']['p50_ms']) for k,v in d.items()})"
for r in 1 2 3; do for pp in 1 3; do
  COA_PRE_PRIO=$pp timeout -k 10 120 python bench.py --steps 40 --no-cpu-baseline --no-secondary > gpurun_out/ab_pp${pp}_r$r.json 2>> gpurun_out/ab.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ab_pp${pp}_r$r.json'));print('prio=$pp', d['value'], d['kernel_ms'], d['verdicts_ok'])"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-secondary --steps 20 > gpurun_out/bench_prof.json 2> gpurun_out/prof.err || { tail -20 gpurun_out/prof.err; exit 1; }
for f in $(find gpurun_out/prof -name "*kernel_stats.csv"); do head -8 "$f"; done
