#!/bin/bash
# GPU call: config-5 probes (1M pods, whole Solve; then again with the phase split)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/c5_probe.py 1000000 > gpurun_out/c5_1m.json 2> gpurun_out/c5_1m.err || { tail -20 gpurun_out/c5_1m.err; exit 1; }
cat gpurun_out/c5_1m.json
KP_TIMING=1 REPS=1 timeout -k 10 300 python -u tools/c5_probe.py 1000000 > gpurun_out/c5_1m_t.json 2> gpurun_out/c5_1m_t.err || { tail -20 gpurun_out/c5_1m_t.err; exit 1; }
cat gpurun_out/c5_1m_t.json
