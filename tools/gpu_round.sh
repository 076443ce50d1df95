#!/bin/bash
# One GPU call: gpu parity tests, default bench, rocprofv3 kernel stats of the bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed rc=$?"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 3 --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || { echo "rocprof failed rc=$?"; tail -30 gpurun_out/bench_prof.err; exit 1; }
find gpurun_out/prof -name '*stats*'
