cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
for cfg in "256 256" "256 64" "256 128" "128 256" "64 64" "256 256"; do
  set -- $cfg
  COA_PRE_BLOCK=$1 COA_MAIN_BLOCK=$2 timeout -k 10 120 python bench.py --no-cpu-baseline --no-secondary --steps 40 > gpurun_out/ab_$1_$2.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab_$1_$2.json'));print('pre $1 main $2', d['value'], d['kernel_ms'], d['verdicts_ok'])"
done
