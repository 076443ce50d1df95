#!/bin/bash
# GPU call: reserved-offering launch parity + the launch / filter / Solve parity suites + a quick bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_reserved_offerings.py \
  tests/test_gpu_launch.py tests/test_filters_golden.py tests/test_gpu_parity.py tests/test_ice_update.py > gpurun_out/pytest_reserved.log 2>&1 \
  || { tail -60 gpurun_out/pytest_reserved.log; exit 1; }
tail -3 gpurun_out/pytest_reserved.log
timeout -k 10 200 python -u bench.py --quick --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/q.json 2> gpurun_out/q.err || { tail -20 gpurun_out/q.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/q.json')); print('kernel_ms', d['solve_kernel_ms'], 'step_ms', d['ms_per_step'])"
