#!/bin/bash
# The whole GPU test suite + smoke, the bench lines with a rocprof of the default bench, and a rocprof of the one-rank
# FSDP bench -> gpurun_out/$TAG/
set -o pipefail
T=${TAG:-r4x}
O=gpurun_out/$T
TAG=$T bash tools/gpu_r4_tests.sh
rc=$?
case $rc in 0|1) ;; *) echo "tests rc=$rc: stopping"; exit $rc ;; esac
TAG=$T PROF=1 bash tools/gpu_r4_bench.sh || exit $?
export TMPDIR=/tmp
timeout -k 10 300 env GPT2MI_FORCE_COLLECTIVES=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29591 \
  rocprofv3 --kernel-trace --stats -d $O/prof_fsdp -o run -- python bench.py --steps 5 --warmup 3 --no-cpu-baseline \
  --parallel fsdp > $O/prof_fsdp.log 2>&1 || exit $?
python tools/rocpd_stats.py $O/prof_fsdp/run_results.db $O/kernel_stats_fsdp.csv && \
  python tools/prof_summary.py $O/kernel_stats_fsdp.csv 8 > $O/summary_fsdp.txt 2>&1; head -40 $O/summary_fsdp.txt
exit $rc
