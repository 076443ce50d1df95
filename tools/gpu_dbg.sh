cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export MALLOC_CHECK_=3
timeout -k 10 300 python -u -m pytest tests/test_ice_update.py -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/dbg1.log 2>&1; echo "rc1=$?"
tail -5 gpurun_out/dbg1.log
