#!/bin/bash
# k_pre_halve role timing (rocprofv3 kernel trace): all roles, decompression
# roles only (COA_PRE_DIAG=4), hash/halving role only (COA_PRE_DIAG=2).
# COA_PRE_DIAG is read only by a library whose coa_halved.hip was compiled with
# -DCOA_PRE_DIAG_BUILD (release builds ignore it): add that flag to COMMON in
# xrpl-coa-prototype_amd/build.py for the run, then rebuild without it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
for diag in 0 4 2; do
  COA_PRE_DIAG=$diag timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/roles_$diag -o run --output-format csv \
    -- python3 tools/inflight_probe.py 65536 20 > gpurun_out/roles_$diag.jsonl 2>&1 || exit 1
  f=$(find gpurun_out/roles_$diag -name "*kernel_stats.csv" | head -1)
  echo "diag $diag: $(grep -h '"k_pre_halve"' $f | cut -d, -f1-4)"
done
