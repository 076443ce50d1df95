#!/bin/bash
# A/B of solve-kernel variants: per-phase profile of configs ${PHASES:-2 3} under each env setting in $VARIANTS
# (space-separated VAR=value, "-" = baseline).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
rm -f gpurun_out/ab.json
for v in ${VARIANTS:--}; do
  for c in ${PHASES:-2 3}; do
    if [ "$v" = "-" ]; then
      timeout -k 10 200 python -u tools/profile_solve.py $c > gpurun_out/ab_one.json 2>> gpurun_out/ab.err || exit $?
    else
      timeout -k 10 200 env $v python -u tools/profile_solve.py $c > gpurun_out/ab_one.json 2>> gpurun_out/ab.err || exit $?
    fi
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_one.json')); d['variant']='$v'; print(json.dumps(d))" >> gpurun_out/ab.json
  done
done
cat gpurun_out/ab.json
