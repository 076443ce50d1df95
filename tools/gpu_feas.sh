#!/bin/bash
# GPU call: the feasibility path's parity tests, its timing (with / without the cheapest stream), then the rocprof
# kernel stats and the FETCH/WRITE PMC passes of the quick bench (config 2 + feasibility).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_tests.sh tests/test_filters_golden.py tests/test_reserved_offerings.py tests/test_template_table.py "tests/test_gpu_parity.py" || exit $?
timeout -k 10 120 python -u tools/feas_bench.py rows > gpurun_out/feas.json 2> gpurun_out/feas.err || { tail -20 gpurun_out/feas.err; exit 1; }
cat gpurun_out/feas.json
SKIP_TESTS=1 SKIP_BENCH=1 bash tools/gpu_bench_prof.sh
