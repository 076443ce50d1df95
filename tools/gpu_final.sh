#!/bin/bash
# GPU call (round end): full bench, rocprofv3 kernel stats + FETCH/WRITE PMC passes of the quick bench (-> traffic
# json), and the SQ instruction-mix passes over one config-2 Solve (-> latency json).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
SKIP_TESTS=1 bash tools/gpu_bench_prof.sh || exit 1
f=$(find gpurun_out/pmc_fetch -name '*counter_collection.csv' | head -1); w=$(find gpurun_out/pmc_write -name '*counter_collection.csv' | head -1)
python3 tools/pmc_traffic.py "$f" "$w" gpurun_out/traffic.json && cat gpurun_out/traffic.json
s=$(find gpurun_out/prof -name '*kernel_stats.csv' | head -1); cp "$s" gpurun_out/kernel_stats_bench_quick.csv
bash tools/pmc_sq.sh > gpurun_out/pmc_sq_config2.log 2>&1 || { tail -5 gpurun_out/pmc_sq_config2.log; exit 1; }
tail -20 gpurun_out/pmc_sq_config2.log; cat gpurun_out/latency.json
