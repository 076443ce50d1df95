#!/bin/bash
# GPU call: Solve parity (fast lane touched), full-size digests, then config-2 and config-5 phase splits and the
# quick bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
KP_T=700 bash tools/gpu_tests.sh tests/test_gpu_parity.py "tests/test_fullsize_parity.py::test_solve_fullsize" tests/test_chunked_order.py tests/test_gpu_topology.py tests/test_hostname_requirements.py tests/test_reference_scenarios.py tests/test_hostports_volumes.py tests/test_uid_order.py tests/test_ice_update.py || exit $?
KP_LIB=$PWD/tools/fine/libkp.so timeout -k 10 200 python -u tools/profile_solve.py 2 > gpurun_out/c2_fine.json 2> gpurun_out/c2.err || { tail -20 gpurun_out/c2.err; exit 1; }
cat gpurun_out/c2_fine.json
timeout -k 10 200 python -u bench.py --quick --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/quick.json 2> gpurun_out/quick.err || { tail -20 gpurun_out/quick.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/quick.json')); print('config2', d['value'], d['ms_per_step'], d['solve_kernel_ms'], d['feasibility']['kernel_ms'] if 'kernel_ms' in d['feasibility'] else d['feasibility'])"
bash tools/gpu_c5_fine.sh
