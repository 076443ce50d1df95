#!/bin/bash
# GPU call: the fast lane's fine phase probes (FT_FINE build, tools/build_fine.sh) on config 3 (100k pods) and config 5
# (1M pods), plus the production library's config-3 kernel time beside them.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 240 env KP_LIB=tools/fine/libkp.so python -u tools/profile_solve.py 3 > gpurun_out/fine_c3.json 2> gpurun_out/fine_c3.err || { tail -20 gpurun_out/fine_c3.err; exit 1; }
cat gpurun_out/fine_c3.json
timeout -k 10 300 env KP_LIB=tools/fine/libkp.so KP_TIMING=1 REPS=1 python -u tools/c5_probe.py 1000000 > gpurun_out/fine_c5.json 2> gpurun_out/fine_c5.err || { tail -20 gpurun_out/fine_c5.err; exit 1; }
cat gpurun_out/fine_c5.json
