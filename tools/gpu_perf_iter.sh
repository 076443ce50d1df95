#!/bin/bash
# Fast-lane iteration: Solve parity tests, the config-2 phase split (FT_FINE build) and a quick bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp; rm -f gpurun_out/phases_*.json
timeout -k 10 600 python -u -m pytest ${KP_TESTS:-tests/test_gpu_parity.py tests/test_reference_scenarios.py tests/test_hostports_volumes.py} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed rc=$?"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
KP_LIB=$PWD/tools/fine/libkp.so timeout -k 10 200 python -u tools/profile_solve.py 2 > gpurun_out/phases_fine.json 2> gpurun_out/phases.err || exit $?
cat gpurun_out/phases_fine.json
timeout -k 10 300 python -u bench.py --quick > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench_quick.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_quick.json')); print('value', d['value'], 'ms', d['ms_per_step'], 'kernel', d.get('solve_kernel_ms'))"
