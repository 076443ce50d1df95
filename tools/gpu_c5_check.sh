#!/bin/bash
# GPU call: the chunked-order / memo parity tests (full-size digests included), then the interleaved config-5 kernel
# A/B (100k pods, then 1M) against tools/variants/*/libkp.so.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread \
  tests/test_fullsize_parity.py tests/test_chunked_order.py tests/test_gpu_parity.py tests/test_uid_order.py \
  > gpurun_out/c5_tests.log 2>&1 || { tail -40 gpurun_out/c5_tests.log; exit 1; }
tail -2 gpurun_out/c5_tests.log
rm -f gpurun_out/ab_c5.txt
for round in 1 2; do
  for lib in karpenter-provider-aws_amd/libkp.so tools/variants/*/libkp.so; do
    KP_LIB=$PWD/$lib timeout -k 10 200 python -u tools/kernel_time.py 5 > gpurun_out/kt.json 2> gpurun_out/kt.err || { echo "$lib failed"; tail -5 gpurun_out/kt.err; exit 1; }
    echo "$lib config5-100k $(cat gpurun_out/kt.json)" | tee -a gpurun_out/ab_c5.txt
    KP_LIB=$PWD/$lib REPS=1 timeout -k 10 200 python -u tools/c5_probe.py 1000000 > gpurun_out/c5.json 2> gpurun_out/c5.err || { echo "$lib failed"; tail -5 gpurun_out/c5.err; exit 1; }
    echo "$lib config5-1M $(python3 -c 'import json;d=json.load(open("gpurun_out/c5.json"));print(json.dumps({"runs":d["runs"],"fast_bails":d["fast_bails"]}))')" | tee -a gpurun_out/ab_c5.txt
  done
done
