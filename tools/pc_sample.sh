#!/bin/bash
# GPU call: list the PC-sampling configurations, then host-trap PC samples over one config-N Solve (solve_kernel's
# instruction hot spots). usage: pc_sample.sh [config] [pods]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
cfg=${1:-2}; n=${2:-50000}
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pcs_list.txt 2>&1; grep -i -A8 "pc.sampl" gpurun_out/pcs_list.txt | head -40
rm -rf gpurun_out/pcs
timeout -k 10 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
  --pc-sampling-interval 1 --kernel-trace --output-format csv -d gpurun_out/pcs -o run -- \
  python3 tools/solve_once.py "$cfg" "$n" 2 > gpurun_out/pcs.log 2>&1 || { echo "pc sampling rc=$?"; tail -20 gpurun_out/pcs.log; exit 1; }
find gpurun_out/pcs -type f | head
