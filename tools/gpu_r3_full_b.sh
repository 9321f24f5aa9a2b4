#!/bin/bash
# round-end check B: the default bench command, then its kernel trace
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 500 python3 -X faulthandler bench.py > gpurun_out/fb_bench.json 2> gpurun_out/fb_bench.err || { tail -20 gpurun_out/fb_bench.err; exit 1; }
tail -c 600 gpurun_out/fb_bench.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/fb -o run --output-format csv -- python3 bench.py > gpurun_out/fb_prof_bench.json 2> gpurun_out/fb_prof.err || { tail -20 gpurun_out/fb_prof.err; exit 1; }
ls gpurun_out/fb/*
