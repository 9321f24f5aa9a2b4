cd "${GRAFT_REPO_ROOT}" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 5 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_verify.py tests/test_gpu_adversarial.py > gpurun_out/t_il.log 2>&1; tail -2 gpurun_out/t_il.log
grep -q passed gpurun_out/t_il.log && ! grep -q failed gpurun_out/t_il.log || exit 1
for rep in 1 2; do
  for il in 0 1; do
    COA_MAIN_IL=$il timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --steps 10 --warmup 2 --n 2097152 > gpurun_out/ab_big_$il.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ab_big_$il.json'));print('n=2^21 IL=$il', d['value'], d['kernel_ms'], d['verdicts_ok'])"
  done
done
for rep in 1 2; do
  for il in 0 1; do
    COA_MAIN_IL=$il timeout -k 10 120 python bench.py --no-cpu-baseline --no-secondary --steps 40 > gpurun_out/ab_c2_$il.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ab_c2_$il.json'));print('C2 IL=$il', d['value'], d['kernel_ms'], d['verdicts_ok'])"
  done
done
