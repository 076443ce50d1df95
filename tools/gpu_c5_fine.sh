#!/bin/bash
# GPU call: config-5 1M with the fast lane's fine phase split (tools/build_fine.sh library)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
KP_LIB=tools/fine/libkp.so KP_TIMING=1 REPS=1 timeout -k 10 300 python -u tools/c5_probe.py ${C5_PODS:-1000000} > gpurun_out/c5_fine.json 2> gpurun_out/c5_fine.err || { tail -20 gpurun_out/c5_fine.err; exit 1; }
cat gpurun_out/c5_fine.json
