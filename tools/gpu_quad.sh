#!/bin/bash
# GPU call: feasibility parity tests, then the feasibility timing of the in-tree library (and its one-row kernel) and
# every tools/variants/feas_*/libkp.so, twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_tests.sh tests/test_filters_golden.py tests/test_reserved_offerings.py tests/test_gpu_parity.py -k "filter or feas or offering or compatible" || exit $?
for i in 1 2; do
timeout -k 10 200 python -u tools/feas_bench.py quad one=KP_FEAS_ONE_ROW=1 temporal=KP_FEAS_TEMPORAL=1 > gpurun_out/feas_quad.json 2> gpurun_out/feas_quad.err || { tail -20 gpurun_out/feas_quad.err; exit 1; }
cat gpurun_out/feas_quad.json
for lib in tools/variants/feas_*/libkp.so; do
  KP_LIB=$PWD/$lib timeout -k 10 120 python -u tools/feas_bench.py rows > gpurun_out/feas.json 2> gpurun_out/feas.err || { tail -20 gpurun_out/feas.err; exit 1; }
  echo "$lib $(cat gpurun_out/feas.json)"
done
done
