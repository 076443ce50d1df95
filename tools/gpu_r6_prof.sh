#!/bin/bash
# GPU call: the full bench line, then per-leg rocprofv3 passes (tools/prof_leg.py): kernel-trace stats, FETCH_SIZE and
# WRITE_SIZE (separate runs), SQ instruction-mix counters for the consolidation legs; tools/pmc_traffic.py keys the
# traffic by leg. Output under gpurun_out/r6prof/. SKIP_BENCH=1 skips the bench; LEGS overrides the leg list.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r6prof
export TMPDIR=/tmp
O=gpurun_out/r6prof
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -30 $O/bench.err; exit 1; }
  cat $O/bench.json
fi
LEGS=${LEGS:-"solve2 feas_rows feas_compact sweep general"}
for leg in $LEGS; do
  reps=3
  [ "$leg" = sweep ] && reps=1
  [ "$leg" = general ] && reps=1
  rm -rf $O/${leg}_stats $O/${leg}_fetch $O/${leg}_write
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${leg}_stats -o run -- python3 tools/prof_leg.py $leg $reps > $O/${leg}_stats.log 2>&1 || { echo "stats $leg rc=$?"; tail -20 $O/${leg}_stats.log; exit 1; }
  tail -1 $O/${leg}_stats.log
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${leg}_fetch -o run -- python3 tools/prof_leg.py $leg 1 > $O/${leg}_fetch.log 2>&1 || { echo "fetch $leg rc=$?"; tail -20 $O/${leg}_fetch.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${leg}_write -o run -- python3 tools/prof_leg.py $leg 1 > $O/${leg}_write.log 2>&1 || { echo "write $leg rc=$?"; tail -20 $O/${leg}_write.log; exit 1; }
  if [ "$leg" = sweep ] || [ "$leg" = general ]; then
    rm -rf $O/${leg}_sq
    timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_INSTS_BRANCH --output-format csv -d $O/${leg}_sq -o run -- python3 tools/prof_leg.py $leg 1 > $O/${leg}_sq.log 2>&1 || { echo "sq $leg rc=$?"; tail -20 $O/${leg}_sq.log; exit 1; }
  fi
done
python3 tools/pmc_traffic.py $O $O/traffic.json > /dev/null
cat $O/traffic.json
find $O -name '*kernel_stats.csv' | sort
