#!/bin/bash
# GPU call (round-6 close): the whole -m gpu suite and smoke, then the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_full_suite.sh || exit 1
timeout -k 10 800 python -u bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -30 gpurun_out/bench_full.err; exit 1; }
tail -c 300 gpurun_out/bench_full.err
