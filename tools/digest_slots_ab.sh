# GPU session (round 5): the streamed C4 line with 4 vs 8 digest slots
# (COA_QUEUE_DIGEST_SLOTS), alternating, each under its own time limit.
set -o pipefail
mkdir -p gpurun_out/ds
for r in 1 2; do
  for k in 8 4; do
    COA_QUEUE_DIGEST_SLOTS=$k timeout -k 10 240 python bench.py --no-cpu-baseline --sections c4_sha512,c4_stream --c4-batches 1024 > gpurun_out/ds/c4_${k}_$r.json 2> gpurun_out/ds/c4_${k}_$r.err || exit 1
  done
done
