#!/bin/bash
# The registration-under-load tests with the queue's slow-window trace (the
# ENQUEUE stage split by call: pin, h2d, launch, d2h, event) and the
# registration's phase trace, REPS times: which call of a window's enqueue
# stalls while a committee registration builds its combs.  (Not under
# rocprofv3: its tracer faults in CU-masked stream creation, DESIGN.md.)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
  COA_QUEUE_TRACE_SLOW_US=${SLOW_US:-2000} COA_REGISTER_TRACE=1 timeout -k 10 300 \
    python3 -m pytest tests/test_gpu_recovery.py -m gpu -s -q -k "register" --timeout 200 \
    > gpurun_out/regtrace_${TAG:-x}_$rep.log 2>&1
  grep -E "slow window|coa_committee_register|passed|failed" gpurun_out/regtrace_${TAG:-x}_$rep.log | cut -c1-260
done
