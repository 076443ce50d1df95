#!/bin/bash
# Instruction-mix PMC pass over one config-2 Solve (solve_kernel): SQ counters (<= 8 per pass) + I-cache.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/pmc_sq gpurun_out/pmc_ic
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_INSTS_BRANCH --output-format csv -d gpurun_out/pmc_sq -o run -- python3 tools/solve_once.py 2 50000 1 > gpurun_out/pmc_sq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_MISSES SQ_INSTS_SMEM SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM --output-format csv -d gpurun_out/pmc_ic -o run -- python3 tools/solve_once.py 2 50000 1 > gpurun_out/pmc_ic.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(float)
for f in glob.glob('gpurun_out/pmc_*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'solve_kernel' in r['Kernel_Name']:
            acc[r['Counter_Name']] += float(r['Counter_Value'])
pops = 50000  # one launch
for k, v in sorted(acc.items()):
    print(f"{k:22s} {v:16.0f} per_pop {v / pops:10.1f}")
# the latency roofline bench.py reads (profiles/latency.json): SQ cycle counters count 4-cycle units summed over the
# workgroup's waves (SQ_WAVE_CYCLES per pod = the measured wall cycles per pod), so the issue floor is 4 x ACTIVE_INST_ANY
import json
ins = sum(acc.get(k, 0) for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_INSTS_SMEM",
                                  "SQ_INSTS_BRANCH")) / pops
json.dump({"issue_cycles_per_pod": round(4 * acc["SQ_ACTIVE_INST_ANY"] / pops, 1), "instructions_per_pod": round(ins, 1),
           "wave_cycles_per_pod": round(4 * acc["SQ_WAVE_CYCLES"] / pops / max(1, acc.get("SQ_WAVES", 4)) , 1),
           "wait_cycles_per_pod": round(4 * acc["SQ_WAIT_ANY"] / pops, 1),
           "source": "tools/pmc_sq.sh: rocprofv3 --pmc SQ counters over one config-2 Solve (50k pods)"},
          open("gpurun_out/latency.json", "w"), indent=1)
PY
