#!/bin/bash
# GPU call: selected -m gpu tests (args: pytest selectors), one pytest process under a time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 ${KP_T:-600} python -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_sel.log | tail -40
[ $rc -ne 0 ] && tail -60 gpurun_out/pytest_sel.log
exit $rc
