#!/bin/bash
# GPU call: the full bench line of the in-tree library and of each tools/variants/*/libkp.so (every leg compared).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for lib in karpenter-provider-aws_amd/libkp.so tools/variants/*/libkp.so; do
  n=$(echo $lib | tr '/' '_')
  KP_LIB=$PWD/$lib timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/b_$n.json 2> gpurun_out/b_$n.err || { echo "$lib failed"; tail -5 gpurun_out/b_$n.err; exit 1; }
  python3 - gpurun_out/b_$n.json $lib <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
c = d["configs"]
print(sys.argv[2], "c2", d["solve_kernel_ms"], "feas", d["feasibility"]["kernel_ms"],
      " ".join(f"{k} {v.get('solve_kernel_ms')}" for k, v in c.items()),
      "cons", d["consolidation"]["value"], "gen", d["consolidation_general"]["value"])
PY
done
