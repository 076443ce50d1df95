#!/bin/bash
# Instruction-mix / stall PMC passes over the feasibility leg (feasibility_quad_kernel / feasibility_bits_kernel, 50k distinct rows, one
# warm-up + FEAS_REPS launches), one pass per counter group.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp FEAS_CHEAPEST_ONLY=1 FEAS_REPS=2
rm -rf gpurun_out/pmcf_*
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmcf_sq -o run -- python3 tools/feas_bench.py rows > gpurun_out/pmcf_sq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA --output-format csv -d gpurun_out/pmcf_sq2 -o run -- python3 tools/feas_bench.py rows > gpurun_out/pmcf_sq2.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(float); n = collections.defaultdict(set)
for f in glob.glob('gpurun_out/pmcf_*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'feasibility_' in r['Kernel_Name'] and 'kernel(' in r['Kernel_Name']:
            acc[r['Counter_Name']] += float(r['Counter_Value'])
            n[r['Counter_Name']].add(r.get('Dispatch_Id', r.get('Correlation_Id', '')))
for k, v in sorted(acc.items()):
    d = max(1, len(n[k]))
    print(f"{k:22s} launches {d:3d} per_launch {v / d:16.0f} per_row {v / d / 50000:10.1f}")
PY
