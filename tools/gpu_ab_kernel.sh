#!/bin/bash
# GPU call: solve_kernel time of config 2 (and config 3 with AB_C3=1) for the in-tree library and every
# tools/variants/*/libkp.so (tools/build_commit_variant.sh / build_variant.sh), interleaved over 3 rounds on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp; rm -f gpurun_out/ab_kernel.txt
for round in 1 2 3; do
  for lib in karpenter-provider-aws_amd/libkp.so tools/variants/*/libkp.so; do
    for cfg in ${AB_CFGS:-2}; do
      KP_LIB=$PWD/$lib timeout -k 10 200 python -u tools/kernel_time.py $cfg > gpurun_out/kt.json 2> gpurun_out/kt.err || { echo "$lib failed"; tail -5 gpurun_out/kt.err; exit 1; }
      echo "$lib config$cfg $(cat gpurun_out/kt.json)" | tee -a gpurun_out/ab_kernel.txt
    done
  done
done
