#!/bin/bash
# Quick config-2 bench of every built variant (tools/variants/*/libkp.so) and of the in-tree library, interleaved twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp; rm -f gpurun_out/variants.txt
for round in 1 2; do
  for lib in karpenter-provider-aws_amd/libkp.so tools/variants/*/libkp.so; do
    KP_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --quick --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/v.json 2> gpurun_out/v.err || { echo "$lib failed"; tail -5 gpurun_out/v.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/v.json')); print(sys.argv[1], 'kernel_ms', d['solve_kernel_ms'], 'step_ms', d['ms_per_step'], 'alg_bytes', d['roofline']['algorithmic_bytes_per_launch'])" $lib | tee -a gpurun_out/variants.txt
  done
done
