# Round-mix tail probe (round 5): the c4_stream and queue_round_mix bench
# sections three times in fresh processes with slow-window tracing
# (COA_QUEUE_TRACE_SLOW_US), each under its own time limit
# (profiles/r05_round_mix_rate5_probe.jsonl).
set -o pipefail
mkdir -p gpurun_out/qmix
for i in 1 2 3; do
  COA_QUEUE_TRACE_SLOW_US=3000 timeout -k 10 240 python bench.py --no-cpu-baseline --sections c4_stream,queue_round_mix > gpurun_out/qmix/run$i.json 2> gpurun_out/qmix/run$i.err || exit 1
  echo "run $i done"
done
