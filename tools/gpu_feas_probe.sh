#!/bin/bash
# GPU call: feasibility variants (tools/feas_bench.py) + one SQ PMC pass per kernel variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/feas_bench.py global=KP_FEAS_GLOBAL=1 lds noprice=KP_FEAS_NO_PRICE=1 nokeys=KP_FEAS_NO_KEYS=1 nores=KP_FEAS_NO_RES=1 b128=KP_FEAS_BLOCKS=128 b512=KP_FEAS_BLOCKS=512 > gpurun_out/feas_probe.json 2> gpurun_out/feas_probe.err || { tail -20 gpurun_out/feas_probe.err; exit 1; }
cat gpurun_out/feas_probe.json
rm -rf gpurun_out/pmcfe_*
for v in lds global; do
  envs=""; [ $v = global ] && envs="KP_FEAS_GLOBAL=1"
  FEAS_REPS=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmcfe_${v}_a -o run -- python3 tools/feas_bench.py "x=$envs" > gpurun_out/pmcfe_${v}_a.log 2>&1 || exit $?
  FEAS_REPS=1 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/pmcfe_${v}_b -o run -- python3 tools/feas_bench.py "x=$envs" > gpurun_out/pmcfe_${v}_b.log 2>&1 || exit $?
done
python3 - <<'PY'
import csv, glob, collections
for v in ("lds", "global"):
    acc = collections.defaultdict(list)
    for f in glob.glob(f'gpurun_out/pmcfe_{v}_*/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if 'feasibility' in r['Kernel_Name'] and int(r.get('Grid_Size', 0) or 0) >= 0:
                acc[(r['Counter_Name'], r['Dispatch_Id'])].append(float(r['Counter_Value']))
    per = collections.defaultdict(list)
    for (c, d), vals in acc.items():
        per[c].append(sum(vals))
    print(v, {c: round(max(x) / 50000, 1) for c, x in sorted(per.items())})
PY
