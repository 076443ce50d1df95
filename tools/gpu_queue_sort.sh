#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_topology.py \
  tests/test_reference_scenarios.py tests/test_fullsize_parity.py tests/test_pod_antiaffinity.py > gpurun_out/pytest_qs.log 2>&1 || { tail -40 gpurun_out/pytest_qs.log; exit 1; }
tail -1 gpurun_out/pytest_qs.log
for round in 1 2; do
  for lib in karpenter-provider-aws_amd/libkp.so tools/variants/base/libkp.so; do
    KP_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --quick --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/v.json 2> gpurun_out/v.err || { tail -5 gpurun_out/v.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/v.json')); print(sys.argv[1], 'kernel_ms', d['solve_kernel_ms'], 'step_ms', d['ms_per_step'], 'prep_ms', d['per_solve_prepare_ms'])" $lib
  done
done
