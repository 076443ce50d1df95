set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
KP_C5_PODS=${KP_C5_PODS:-1000000} timeout -k 10 400 python -u tools/probe_configs.py ${PROBE:-2 3 5} > gpurun_out/probe.json 2> gpurun_out/probe.err; rc=$?
cat gpurun_out/probe.json; tail -5 gpurun_out/probe.err; exit $rc
