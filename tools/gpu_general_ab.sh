#!/bin/bash
# GPU call: the general-path parity tests, then the 10k-node general leg (100 prefixes + 100k subsets) for the in-tree
# library and tools/variants/*/libkp.so, interleaved over 3 rounds on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_sim_general.py \
  tests/test_reserved_consolidation.py tests/test_cancel.py tests/test_e2e_suites.py "tests/test_fullsize_parity.py::test_general_10000" \
  "tests/test_fullsize_parity.py::test_general_fullsize" > gpurun_out/gen_tests.log 2>&1 || { tail -40 gpurun_out/gen_tests.log; exit 1; }
tail -1 gpurun_out/gen_tests.log
rm -f gpurun_out/ab_general.txt
for round in 1 2 3; do
  for lib in karpenter-provider-aws_amd/libkp.so tools/variants/*/libkp.so; do
    KP_LIB=$PWD/$lib timeout -k 10 200 python -u tools/general_scale.py 10000 100000 > gpurun_out/gs.out 2> gpurun_out/gs.err || { echo "$lib failed"; tail -5 gpurun_out/gs.err; exit 1; }
    echo "$lib $(tail -1 gpurun_out/gs.out)" | tee -a gpurun_out/ab_general.txt
  done
done
