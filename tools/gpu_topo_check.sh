#!/bin/bash
# GPU call: the topology-path parity tests (device == oracle), then the interleaved kernel A/B of configs 2 and 3
# against tools/variants/*/libkp.so (tools/gpu_ab_kernel.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_topology.py tests/test_pod_antiaffinity.py tests/test_hostname_requirements.py \
  tests/test_prefer_no_schedule.py tests/test_sim_general.py tests/test_e2e_suites.py \
  "tests/test_fullsize_parity.py" > gpurun_out/topo_tests.log 2>&1 || { tail -40 gpurun_out/topo_tests.log; exit 1; }
tail -2 gpurun_out/topo_tests.log
AB_CFGS="${AB_CFGS:-2 3}" bash tools/gpu_ab_kernel.sh
