#!/bin/bash
# round 3: counter profile of the C2 verify call on this build (three
# separate --pmc passes, as MI355X_MICROARCH.md prescribes) -> profiles JSON
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -T -d gpurun_out/vp/pmc_SQ -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-secondary --steps 3 --warmup 1 > gpurun_out/vp_sq.json 2> gpurun_out/vp_sq.err || { tail -30 gpurun_out/vp_sq.err; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $c -T -d gpurun_out/vp/pmc_$c -o run --output-format csv \
      -- python3 bench.py --no-cpu-baseline --no-secondary --steps 3 --warmup 1 > gpurun_out/vp_$c.json 2> gpurun_out/vp_$c.err || { tail -30 gpurun_out/vp_$c.err; exit 1; }
done
python3 tools/pmc_verify.py gpurun_out/vp 65536 gpurun_out/r03_verify_pmc.json && echo "verify_pmc ok"
timeout -k 10 -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -T -d gpurun_out/vpw/pmc_SQ -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-secondary --steps 3 --warmup 1 > gpurun_out/vpw_sq.json 2> gpurun_out/vpw_sq.err || { tail -30 gpurun_out/vpw_sq.err; exit 1; }
echo waits ok
