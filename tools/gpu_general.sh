#!/bin/bash
# GPU call: the general-path consolidation leg alone, with the host phase split (KP_HOST_TIMING)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
KP_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --only-general ${GEN_ARGS:-} > gpurun_out/general.json 2> gpurun_out/general.err || { tail -20 gpurun_out/general.err; exit 1; }
cat gpurun_out/general.json
grep "kp general" gpurun_out/general.err | tail -5
