#!/bin/bash
# GPU call: feasibility parity tests, feasibility variants (tools/feas_bench.py), then the SQ PMC passes behind the
# bench line's latency roofline (tools/pmc_sq.sh -> gpurun_out/latency.json).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_reserved_offerings.py -m gpu -x -q -k "feas or compatible or filter" --timeout 120 --timeout-method thread > gpurun_out/pytest_feas.log 2>&1 || { tail -30 gpurun_out/pytest_feas.log; exit 1; }
tail -1 gpurun_out/pytest_feas.log
timeout -k 10 300 python3 -u tools/feas_bench.py nt temporal=KP_FEAS_TEMPORAL=1 b2048=KP_FEAS_BLOCKS=2048 b1024=KP_FEAS_BLOCKS=1024 > gpurun_out/feas_probe.json 2> gpurun_out/feas_probe.err || { tail -20 gpurun_out/feas_probe.err; exit 1; }
cat gpurun_out/feas_probe.json
bash tools/pmc_sq.sh && cat gpurun_out/latency.json
