#!/bin/bash
# Fast-lane phase split (FT_FINE diagnostic build in tools/fine/libkp.so) of config 2, then the coarse split of 2 and 5.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp; rm -f gpurun_out/phases_*.json
KP_LIB=$PWD/tools/fine/libkp.so timeout -k 10 200 python -u tools/profile_solve.py 2 > gpurun_out/phases_fine.json 2> gpurun_out/phases.err || exit $?
for c in ${PHASES:-2 5}; do timeout -k 10 200 python -u tools/profile_solve.py $c > gpurun_out/phases_c$c.json 2>> gpurun_out/phases.err || exit $?; done
cat gpurun_out/phases_*.json
