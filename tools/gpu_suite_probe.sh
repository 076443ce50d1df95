#!/bin/bash
# GPU call: the whole -m gpu suite, then full-size config probes (args: configs, default 2 3 5).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
fi
timeout -k 10 400 python -u tools/probe_configs.py ${@:-2 3 5} > gpurun_out/probe.json 2> gpurun_out/probe.err || { tail -30 gpurun_out/probe.err; exit 1; }
cat gpurun_out/probe.json
