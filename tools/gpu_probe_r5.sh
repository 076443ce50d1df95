set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 5 60 tools/micro/lat > gpurun_out/micro_lat.txt 2>&1 && timeout -k 5 60 tools/micro/issue > gpurun_out/micro_issue.txt 2>&1 && cat gpurun_out/micro_lat.txt gpurun_out/micro_issue.txt || exit 1
timeout -k 10 200 python -u tools/kernel_time.py 3 > gpurun_out/kt3.json 2> gpurun_out/kt3.err || { tail -5 gpurun_out/kt3.err; exit 1; }
cat gpurun_out/kt3.json
KP_HOST_TIMING=1 timeout -k 10 200 python -u tools/solve_once.py 3 100000 1 > gpurun_out/so3.txt 2>&1 || { tail -5 gpurun_out/so3.txt; exit 1; }
grep "kp compile" gpurun_out/so3.txt | tail -12
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -k "topology or affinity or hostname or fullsize or general or prefer" --timeout 300 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?; tail -3 gpurun_out/pt.log; exit $rc
