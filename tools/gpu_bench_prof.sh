#!/bin/bash
# GPU call: gpu tests, full bench, rocprofv3 kernel stats of a quick bench, and separate PMC passes
# (FETCH_SIZE, WRITE_SIZE) for the HBM traffic of solve_kernel and feasibility_kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench rc=$?"; tail -30 gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --quick --steps 3 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { echo "rocprof rc=$?"; tail -20 gpurun_out/prof.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --quick --steps 3 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_fetch.log 2>&1 || { echo "pmc fetch rc=$?"; tail -20 gpurun_out/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --quick --steps 3 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_write.log 2>&1 || { echo "pmc write rc=$?"; tail -20 gpurun_out/pmc_write.log; exit 1; }
find gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write -name '*.csv' | head -20
