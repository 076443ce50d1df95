#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_reserved_offerings.py \
  tests/test_ice_update.py > gpurun_out/pytest_reserved.log 2>&1 || { tail -60 gpurun_out/pytest_reserved.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/pytest_reserved.log | tail -20; tail -1 gpurun_out/pytest_reserved.log
