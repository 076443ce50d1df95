#!/bin/bash
# GPU call: feasibility grid sweep, config-5 1M probe (whole Solve, then with the phase split), then the whole -m gpu
# suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python -u tools/feas_bench.py def blk512=KP_FEAS_BLOCKS=512 blk1024=KP_FEAS_BLOCKS=1024 blk2048=KP_FEAS_BLOCKS=2048 blk4096=KP_FEAS_BLOCKS=4096 > gpurun_out/feas_blk.json 2> gpurun_out/feas_blk.err || { tail -20 gpurun_out/feas_blk.err; exit 1; }
cat gpurun_out/feas_blk.json
bash tools/gpu_c5.sh || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -20
exit $rc
