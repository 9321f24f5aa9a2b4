#!/bin/bash
# round-end check A: the whole GPU suite and smoke()
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests/ > gpurun_out/full_tests.log 2>&1; rc=$?
tail -5 gpurun_out/full_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
