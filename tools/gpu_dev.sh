#!/bin/bash
# Development GPU call: parity tests, then per-phase profile and full-size probes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -2 gpurun_out/pytest_gpu.log
rm -f gpurun_out/phases.json
for c in ${PHASES:-2 3 5}; do timeout -k 10 200 python -u tools/profile_solve.py $c >> gpurun_out/phases.json 2>> gpurun_out/phases.err || exit $?; done
cat gpurun_out/phases.json
