#!/bin/bash
# GPU call: feasibility timing (50k distinct rows, with / without the cheapest stream) of the in-tree library and of
# every tools/variants/feas_*/libkp.so, interleaved twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp; rm -f gpurun_out/feas_var.txt
for round in 1 2; do
  for lib in karpenter-provider-aws_amd/libkp.so tools/variants/feas_*/libkp.so; do
    KP_LIB=$PWD/$lib timeout -k 10 120 python -u tools/feas_bench.py rows > gpurun_out/feas.json 2> gpurun_out/feas.err || { tail -20 gpurun_out/feas.err; exit 1; }
    echo "$lib $(cat gpurun_out/feas.json)" | tee -a gpurun_out/feas_var.txt
  done
done
