#!/bin/bash
# Kernel iteration: GPU parity (Solve) tests, then the per-phase profile of configs 2 and 5 (KP_TIMING).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; rm -f gpurun_out/phases.json
timeout -k 10 600 python -u -m pytest ${KP_TESTS:-tests/test_gpu_parity.py tests/test_gpu_topology.py tests/test_reference_scenarios.py} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed rc=$?"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for c in ${PHASES:-2 5}; do timeout -k 10 200 python -u tools/profile_solve.py $c >> gpurun_out/phases.json 2>> gpurun_out/phases.err || exit $?; done
cat gpurun_out/phases.json
