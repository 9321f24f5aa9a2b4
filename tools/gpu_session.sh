#!/bin/bash
# One parameterised GPU-session script (it replaces round 3's 26 one-off
# tools/gpu_r3_*.sh compositions): tools/gpu_session.sh <step> [args]
#   env              box environment relevant to HIP queues -> gpurun_out/${R:-r6}_env.txt
#   hwq              hardware-queue probe matrix (tools/hwq_probe) -> ${R:-r6}_hwq.jsonl
#   tests [ARGS]     the GPU test suite (pytest -m gpu ARGS) -> ${R:-r6}_tests.log
#   bench HQ TAG ARGS  bench.py ARGS with GPU_MAX_HW_QUEUES=HQ ("-": as the box
#                    has it) -> ${R:-r6}_bench_TAG.json
#   ab ENVS [N]      same-box A/B of runtime switches on the C2 line
#                    (tools/ab_env.sh; ENVS="name=VAR=value ... default")
#   probe SCRIPT ARGS  a tools/ probe under its own time limit
#   pmcsec SECTION TAG KERNEL...  counter passes of one bench section
#   kstats TAG ARGS  rocprofv3 kernel trace + stats of bench.py ARGS
#   smoke            __graft_entry__.smoke()
# (kernel stats and counter passes: tools/gpu_round.sh prof | verifypmc)
# Every GPU step runs under its own timeout; the script stops at the first
# failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
step=$1
shift
case "$step" in
  env)
    env | grep -E '^(GPU_|HIP_|HSA_|ROC|AMD_|OMP_)' | sort > gpurun_out/${R:-r6}_env.txt
    (nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null) >> gpurun_out/${R:-r6}_env.txt
    ;;
  hwq)
    out=gpurun_out/${R:-r6}_hwq.jsonl
    : > $out
    for hq in unset 4 8; do
      for kind in plain cumask hi lo; do
        for bg in 0 3; do
          if [ $hq = unset ]; then
            timeout -k 5 30 env -u GPU_MAX_HW_QUEUES tools/hwq_probe $kind 8 $bg >> $out || exit 1
          else
            GPU_MAX_HW_QUEUES=$hq timeout -k 5 30 tools/hwq_probe $kind 8 $bg >> $out || exit 1
          fi
        done
      done
    done
    ;;
  bench)
    hq=$1
    tag=$2
    shift 2
    if [ "$hq" = "-" ]; then
      timeout -k 10 400 python -u bench.py "$@" > gpurun_out/${R:-r6}_bench_$tag.json 2> gpurun_out/${R:-r6}_bench_$tag.err || exit 1
    else
      GPU_MAX_HW_QUEUES=$hq timeout -k 10 400 python -u bench.py "$@" > gpurun_out/${R:-r6}_bench_$tag.json 2> gpurun_out/${R:-r6}_bench_$tag.err || exit 1
    fi
    ;;
  tests)
    timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/${R:-r6}_tests.log 2>&1 || exit 1
    ;;
  ab)
    ENVS="$1" N=${2:-65536} REPS=${REPS:-3} bash tools/ab_env.sh || exit 1
    ;;
  probe)
    script=$1
    shift
    timeout -k 10 300 python -u "tools/$script" "$@" || exit 1
    ;;
  pmcsec)
    # counter passes of one bench section -> tools/pmc_kernels.py summary:
    # tools/gpu_session.sh pmcsec SECTION TAG KERNEL...
    sec=$1
    tag=$2
    shift 2
    d=gpurun_out/pmc_$tag
    rm -rf $d
    for pass in "SQ:SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
                "WAIT:SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY SQ_INSTS_LDS" \
                "FETCH_SIZE:FETCH_SIZE" "WRITE_SIZE:WRITE_SIZE"; do
      name=${pass%%:*}
      ctrs=${pass#*:}
      timeout -k 10 -s KILL 300 rocprofv3 --pmc $ctrs --kernel-trace -d $d/pmc_$name -o run --output-format csv \
        -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --settle-s 0 --sections $sec \
        > $d.$name.json 2> $d.$name.err || { tail -20 $d.$name.err; exit 1; }
    done
    python3 tools/pmc_kernels.py $d gpurun_out/pmc_$tag.json "$@" || exit 1
    ;;
  pmcx)
    # raw counter passes of one bench section: tools/gpu_session.sh pmcx
    # SECTION TAG "NAME:CTR CTR ..." ... -> medians per (kernel, grid)
    sec=$1
    tag=$2
    shift 2
    d=gpurun_out/pmcx_$tag
    rm -rf $d
    for pass in "$@"; do
      name=${pass%%:*}
      ctrs=${pass#*:}
      timeout -k 10 -s KILL 300 rocprofv3 --pmc $ctrs --kernel-trace -d $d/pmc_$name -o run --output-format csv \
        -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --settle-s 0 --sections $sec \
        > $d.$name.json 2> $d.$name.err || { tail -20 $d.$name.err; exit 1; }
    done
    python3 tools/pmc_kernels.py --raw $d gpurun_out/pmcx_$tag.json || exit 1
    ;;
  kstats)
    # per-kernel durations of a bench run: tools/gpu_session.sh kstats TAG ARGS
    # (runtime switches come in through the environment)
    tag=$1
    shift
    rm -rf gpurun_out/kstats_$tag
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kstats_$tag -o run --output-format csv \
      -- python3 bench.py --no-cpu-baseline --settle-s 0 "$@" > gpurun_out/kstats_$tag.json \
      2> gpurun_out/kstats_$tag.err || { tail -20 gpurun_out/kstats_$tag.err; exit 1; }
    ;;
  smoke)
    timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
    ;;
  *)
    echo "unknown step $step" >&2
    exit 2
    ;;
esac
