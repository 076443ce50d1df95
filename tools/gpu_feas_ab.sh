#!/bin/bash
# GPU call: feasibility parity tests on the in-tree library, then the feasibility timing of the in-tree library
# against tools/variants/feas_old, then the config-2 / config-5 A/B (tools/gpu_ab.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_tests.sh tests/test_filters_golden.py tests/test_reserved_offerings.py tests/test_template_table.py tests/test_gpu_parity.py -k "filter or feas or offering or template" || exit $?
for round in 1 2; do
  for lib in karpenter-provider-aws_amd/libkp.so tools/variants/feas_old/libkp.so; do
    KP_LIB=$PWD/$lib timeout -k 10 120 python -u tools/feas_bench.py rows > gpurun_out/feas.json 2> gpurun_out/feas.err || { tail -20 gpurun_out/feas.err; exit 1; }
    echo "$lib $(cat gpurun_out/feas.json)" | tee -a gpurun_out/feas_ab.txt
  done
done
[ -n "$NO_AB" ] || bash tools/gpu_ab.sh
