#!/bin/bash
# GPU call: the config-4 sweep (tools/prof_leg.py sweep: 1M subsets, one sim_kernel launch) for the in-tree library and
# every tools/variants/*/libkp.so, interleaved over 3 rounds on one box -> gpurun_out/ab_sweep.txt
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp; rm -f gpurun_out/ab_sweep.txt
for round in 1 2 3; do
  for lib in karpenter-provider-aws_amd/libkp.so tools/variants/*/libkp.so; do
    KP_LIB=$PWD/$lib timeout -k 10 200 python -u tools/prof_leg.py ${AB_LEG:-sweep} ${AB_REPS:-1} > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "$lib failed"; tail -5 gpurun_out/ab.err; exit 1; }
    echo "$lib $(cat gpurun_out/ab.json)" | tee -a gpurun_out/ab_sweep.txt
  done
done
