#!/bin/bash
# GPU call: selected -m gpu test files (args), then the quick bench (config 2 + feasibility) under rocprofv3 stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1 || { tail -60 gpurun_out/pytest_quick.log; exit 1; }
  tail -3 gpurun_out/pytest_quick.log
fi
timeout -k 10 300 python -u bench.py --quick --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { tail -30 gpurun_out/bench_quick.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_quick.json'))
print('value', d['value'], 'ms', d['ms_per_step'], 'kernel', d['solve_kernel_ms'])
f=d['feasibility']; print('feas', f['kernel_ms'], f['roofline']['achieved'], f['roofline']['frac'], 'shapes', f['config2_shapes']['kernel_ms'])
"
