#!/bin/bash
# GPU call: the tests touched this round, then the general leg, the config-5 fine probe and the feasibility
# timing + rocprof stats + FETCH/WRITE PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
KP_T=700 bash tools/gpu_tests.sh ${ROUND_TESTS:-tests/test_gpu_parity.py tests/test_fullsize_parity.py tests/test_sim_general.py tests/test_reserved_consolidation.py tests/test_hostname_requirements.py tests/test_chunked_order.py tests/test_filters_golden.py tests/test_reserved_offerings.py tests/test_template_table.py} || exit $?
bash tools/gpu_general.sh || exit $?
bash tools/gpu_c5_fine.sh || exit $?
timeout -k 10 120 python -u tools/feas_bench.py rows > gpurun_out/feas.json 2> gpurun_out/feas.err || { tail -20 gpurun_out/feas.err; exit 1; }
cat gpurun_out/feas.json
SKIP_TESTS=1 SKIP_BENCH=1 bash tools/gpu_bench_prof.sh || exit $?
bash tools/gpu_c3.sh
