#!/bin/bash
# One GPU call: the -m gpu parity suite, then a quick bench (config 2 + feasibility).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${KP_TESTS:-tests} -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed rc=$?"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --quick ${KP_BENCH_ARGS:-} > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench_quick.err; exit 1; }
cat gpurun_out/bench_quick.json
