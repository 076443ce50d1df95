#!/bin/bash
# GPU call: config-3 phase splits: coarse (product build), the fast lane's fine split, the existing-node scan split
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python -u tools/profile_solve.py 3 > gpurun_out/c3_coarse.json 2> gpurun_out/c3.err || { tail -20 gpurun_out/c3.err; exit 1; }
KP_LIB=$PWD/tools/fine/libkp.so timeout -k 10 200 python -u tools/profile_solve.py 3 > gpurun_out/c3_fine.json 2>> gpurun_out/c3.err || { tail -20 gpurun_out/c3.err; exit 1; }
EX_DIAG=1 KP_LIB=$PWD/tools/variants/exdiag/libkp.so timeout -k 10 200 python -u tools/profile_solve.py 3 > gpurun_out/c3_ex.json 2>> gpurun_out/c3.err || { tail -20 gpurun_out/c3.err; exit 1; }
cat gpurun_out/c3_coarse.json gpurun_out/c3_fine.json gpurun_out/c3_ex.json
