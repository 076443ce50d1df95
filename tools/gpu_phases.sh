set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for c in ${PHASES:-2 3 5}; do timeout -k 10 200 python -u tools/profile_solve.py $c >> gpurun_out/phases.json 2>> gpurun_out/phases.err || exit $?; done
cat gpurun_out/phases.json
