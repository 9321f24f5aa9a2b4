#!/bin/bash
# one uncached verify_batch group (67 votes): p50, then the kernel trace
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 120 python3 tools/msm1_probe.py 67 300 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/msm1 -o run --output-format csv -- python3 tools/msm1_probe.py 67 50 > gpurun_out/msm1.json 2> gpurun_out/msm1.err || { tail -20 gpurun_out/msm1.err; exit 1; }
ls gpurun_out/msm1/*
