#!/bin/bash
# GPU call: the -m gpu suite (stops at the first failure), then the quick bench and the config-2 / burst phase splits.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 400 python -u bench.py --quick --steps 10 > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { tail -20 gpurun_out/bench_quick.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_quick.json')); print('headline', d['value'], d['ms_per_step'], d['roofline']['achieved'])"
KP_LIB=$PWD/tools/fine/libkp.so timeout -k 10 200 python -u tools/profile_solve.py 2 > gpurun_out/c2_fine.json 2> gpurun_out/prof.err || exit 1
cat gpurun_out/c2_fine.json
