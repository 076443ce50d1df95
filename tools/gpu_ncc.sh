#!/bin/bash
# GPU call: config-2 / config-3 kernel time with the failure memo's NodeClaim capacity capped (KP_NCC_CAP), interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp; rm -f gpurun_out/ncc.txt
for round in 1 2; do
  for cap in 0 8192 1024 256; do
    for cfg in ${NCC_CFGS:-2 3}; do
      if [ $cap = 0 ]; then unset KP_NCC_CAP; else export KP_NCC_CAP=$cap; fi
      timeout -k 10 200 python -u tools/kernel_time.py $cfg > gpurun_out/kt.json 2> gpurun_out/kt.err || { tail -5 gpurun_out/kt.err; exit 1; }
      echo "cap=$cap config$cfg $(cat gpurun_out/kt.json)" | tee -a gpurun_out/ncc.txt
    done
  done
done
