#!/bin/bash
# GPU call: feasibility leg (tools/feas_bench.py) for the in-tree library and every tools/variants/*/libkp.so, twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp; rm -f gpurun_out/feas_variants.txt
for round in 1 2; do
  for lib in karpenter-provider-aws_amd/libkp.so tools/variants/*/libkp.so; do
    KP_LIB=$PWD/$lib timeout -k 10 120 python3 -u tools/feas_bench.py x > gpurun_out/fv.json 2> gpurun_out/fv.err || { echo "$lib failed"; tail -5 gpurun_out/fv.err; exit 1; }
    echo "$lib $(cat gpurun_out/fv.json)" | tee -a gpurun_out/feas_variants.txt
  done
done
