#!/bin/bash
# GPU call: the interleaved kernel A/B (tools/gpu_ab_kernel.sh, AB_CFGS) of the in-tree library against
# tools/variants/*, then the in-tree library's parity tests selected by AB_TESTS (a pytest -k expression).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_ab_kernel.sh || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -k "${AB_TESTS:-fullsize or gpu_parity}" --timeout 300 --timeout-method thread > gpurun_out/pt_ab.log 2>&1; rc=$?
tail -3 gpurun_out/pt_ab.log; [ $rc -ne 0 ] && grep -E "FAILED|Error|assert" gpurun_out/pt_ab.log | head -20
exit $rc
