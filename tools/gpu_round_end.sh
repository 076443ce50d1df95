#!/bin/bash
# GPU call (round end): the whole -m gpu suite, then tools/gpu_final.sh (bench, rocprof stats, PMC traffic, SQ mix).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
bash tools/gpu_final.sh
