#!/bin/bash
# Latency-structure PMC pass over one config-2 Solve (solve_kernel): instruction fetches (taken-branch redirects),
# branches, and the VMEM / LDS in-flight levels (level / instructions = average latency in SQ cycles).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
cfg=${1:-2}; n=${2:-50000}
rm -rf gpurun_out/pmc_sq2
timeout -s KILL 120 rocprofv3 --pmc SQ_IFETCH SQ_INSTS_BRANCH SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES --output-format csv -d gpurun_out/pmc_sq2 -o run -- python3 tools/solve_once.py $cfg $n 1 > gpurun_out/pmc_sq2.log 2>&1 || exit $?
python3 - "$n" <<'PY'
import csv, glob, collections, sys
acc = collections.defaultdict(float)
for f in glob.glob('gpurun_out/pmc_sq2/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'solve_kernel' in r['Kernel_Name']:
            acc[r['Counter_Name']] += float(r['Counter_Value'])
pods = int(sys.argv[1])
for k, v in sorted(acc.items()):
    print(f"{k:22s} {v:16.0f} per_pod {v / pods:10.1f}")
if acc.get('SQ_INSTS_VMEM'): print('vmem level/insts', acc['SQ_INST_LEVEL_VMEM'] / acc['SQ_INSTS_VMEM'])
if acc.get('SQ_INSTS_LDS'): print('lds level/insts', acc['SQ_INST_LEVEL_LDS'] / acc['SQ_INSTS_LDS'])
PY
