#!/bin/bash
# Aggregation-queue throughput (tools/queue_probe.c): windows in flight per
# GPU / signatures per request (1 = coa_queue_submit_verify, more =
# coa_queue_submit_verify_many); 2^21 signatures from 8 producers, windows of
# up to 65,536.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
for cfg in ${CFGS:-2/1 1/1 4/1 2/64 4/64 2/1024 4/1024}; do
  slots=${cfg%/*}; group=${cfg#*/}
  COA_QUEUE_SLOTS=$slots timeout -k 10 120 ./tools/queue_probe ${REQS:-2097152} ${PROD:-8} ${MB:-65536} ${DELAY:-200} $group \
    >> gpurun_out/queue_probe.jsonl 2>> gpurun_out/queue_probe.err || exit 1
  tail -1 gpurun_out/queue_probe.jsonl
done
