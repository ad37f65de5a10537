#!/bin/bash
# Round 6: rocprofv3 kernel-trace summaries of the bench step under settings (SIDES="A C", env AB_A / AB_C ...) ->
# gpurun_out/$TAG/summary_<side>.txt (one profiled bench per side, 8 timed steps)
set -o pipefail
O=gpurun_out/${TAG:-r6d}
mkdir -p $O
export TMPDIR=/tmp
for side in ${SIDES:-A B}; do
  v=AB_$side; envs="${!v:-X_AB=$side}"
  for kv in $envs; do export "$kv"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$side -o run -- python bench.py --steps 8 --warmup 3 \
    --no-cpu-baseline ${BENCH_ARGS} > $O/prof_$side.log 2>&1 || exit $?
  for kv in $envs; do unset "${kv%%=*}"; done
  python tools/rocpd_stats.py $O/prof_$side/run_results.db $O/kernel_stats_$side.csv && \
    python tools/prof_summary.py $O/kernel_stats_$side.csv 11 > $O/summary_$side.txt 2>&1 || exit $?
  rm -rf $O/prof_$side
  echo "== $side ($envs)"; head -24 $O/summary_$side.txt; tail -1 $O/summary_$side.txt
done
