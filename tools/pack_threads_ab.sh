# GPU session (round 5): host_e2e (C2/C3 host paths, streamed C3) with 8 vs 16 pack threads
set -o pipefail
mkdir -p gpurun_out/pk
for r in 1 2; do
  for t in 8 16; do
    COA_PACK_THREADS=$t timeout -k 10 300 python bench.py --no-cpu-baseline --sections host_e2e > gpurun_out/pk/he_${t}_$r.json 2> gpurun_out/pk/he_${t}_$r.err || exit 1
  done
done
