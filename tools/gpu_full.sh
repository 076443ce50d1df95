#!/bin/bash
# GPU tests (selection via KP_TESTS), then the default bench; each step under its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${KP_TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed rc=$?"; grep -v "^  File" gpurun_out/pytest_gpu.log | tail -40; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
[ -n "$KP_NO_BENCH" ] && exit 0
timeout -k 10 900 python -u bench.py ${KP_BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
