#!/bin/bash
# GPU call: the feasibility equality tests, then the two feasibility legs for the in-tree library and
# tools/variants/*/libkp.so, interleaved over 3 rounds on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_filters_golden.py -k "filter or feas or compact or golden" > gpurun_out/feas_tests.log 2>&1 || { tail -30 gpurun_out/feas_tests.log; exit 1; }
tail -1 gpurun_out/feas_tests.log
rm -f gpurun_out/ab_feas.txt
for round in 1 2 3; do
  for lib in karpenter-provider-aws_amd/libkp.so tools/variants/*/libkp.so; do
    KP_LIB=$PWD/$lib timeout -k 10 200 python -u tools/feas_ab.py > gpurun_out/fa.json 2> gpurun_out/fa.err || { echo "$lib failed"; tail -5 gpurun_out/fa.err; exit 1; }
    echo "$lib $(cat gpurun_out/fa.json)" | tee -a gpurun_out/ab_feas.txt
  done
done
