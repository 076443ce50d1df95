#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_reserved_offerings.py \
  tests/test_gpu_launch.py tests/test_filters_golden.py > gpurun_out/pytest_reserved.log 2>&1 || { tail -60 gpurun_out/pytest_reserved.log; exit 1; }
tail -2 gpurun_out/pytest_reserved.log
bash tools/gpu_variants.sh
