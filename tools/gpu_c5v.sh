#!/bin/bash
# GPU call: config-5 1M probe, config-2 quick bench, then the whole -m gpu suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
REPS=2 timeout -k 10 300 python -u tools/c5_probe.py 1000000 > gpurun_out/c5_1m.json 2> gpurun_out/c5_1m.err || { tail -20 gpurun_out/c5_1m.err; exit 1; }
cat gpurun_out/c5_1m.json
timeout -k 10 200 python -u bench.py --quick --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/v.json 2> gpurun_out/v.err || { tail -5 gpurun_out/v.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/v.json')); print('config2_kernel_ms', d['solve_kernel_ms'], 'step_ms', d['ms_per_step'], 'feas', d['feasibility']['kernel_ms'])"
[ -n "$NO_SUITE" ] && exit 0
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -20
exit $rc
