#!/bin/bash
# one-group Pippenger p50 at each lane run length (exact route, 67 votes)
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out
for r in 1 2 4 8 16; do
  echo "run=$r"; COA_BATCH_LAT=0 COA_MSM_RUN=$r timeout -k 10 120 python3 tools/msm1_probe.py 67 300 || exit 1
done
