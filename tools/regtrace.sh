#!/bin/bash
# HIP API trace of test_registration_never_holds_a_window_back (the slot
# streams forced CU-masked, as without a profiler): which call of the queue's
# enqueue stalls while a committee-100 registration builds its combs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
rm -rf gpurun_out/regtrace
COA_QUEUE_STREAMS=cumask COA_QUEUE_TRACE_SLOW_US=3000 COA_REGISTER_TRACE=1 timeout -k 10 300 \
  rocprofv3 --hip-trace --kernel-trace -d gpurun_out/regtrace -o run --output-format csv -- \
  python3 -m pytest tests/test_gpu_recovery.py -m gpu -s -q -k "registration_never" --timeout 200 \
  > gpurun_out/regtrace.log 2>&1
rc=$?
python3 - <<'PY'
import csv, glob
rows = []
for p in glob.glob("gpurun_out/regtrace/**/*hip_api_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(p)))
slow = sorted(((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, r["Function"], r["Thread_Id"],
               int(r["Start_Timestamp"])) for r in rows)
print("hip api calls:", len(rows))
for d, f, t, s in slow[-40:]:
    print(f"{d:10.1f} us  {f}  thread {t}  start {s}")
PY
exit $rc
