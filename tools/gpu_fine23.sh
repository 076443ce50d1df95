set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for c in 2 3; do KP_LIB=$PWD/tools/fine/libkp.so timeout -k 10 200 python -u tools/profile_solve.py $c > gpurun_out/phases_fine_c$c.json 2> gpurun_out/phases.err || exit $?; done
cat gpurun_out/phases_fine_c2.json; echo; cat gpurun_out/phases_fine_c3.json
