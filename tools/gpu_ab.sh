#!/bin/bash
# GPU call: A/B of the in-tree library against tools/variants/*: config-2 quick bench and config-5 1M, interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp; rm -f gpurun_out/ab.txt
[ -n "$AB_PRE_TESTS" ] && { bash tools/gpu_tests.sh $AB_PRE_TESTS || exit $?; }
for round in 1 2; do
  for lib in karpenter-provider-aws_amd/libkp.so tools/variants/*/libkp.so; do
    KP_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --quick --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/v.json 2> gpurun_out/v.err || { echo "$lib failed"; tail -5 gpurun_out/v.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/v.json')); print(sys.argv[1], 'config2_kernel_ms', d['solve_kernel_ms'], 'step_ms', d['ms_per_step'])" $lib | tee -a gpurun_out/ab.txt
    if [ -n "$AB_C5" ]; then
      KP_LIB=$PWD/$lib REPS=1 timeout -k 10 200 python -u tools/c5_probe.py 1000000 > gpurun_out/v5.json 2> gpurun_out/v5.err || { echo "$lib c5 failed"; tail -5 gpurun_out/v5.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open('gpurun_out/v5.json')); print(sys.argv[1], 'config5_kernel_ms', d['runs'][0]['kernel_ms'])" $lib | tee -a gpurun_out/ab.txt
    fi
  done
done
