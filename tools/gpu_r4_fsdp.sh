#!/bin/bash
# FSDP changes: the data-parallel / trainer / optimizer GPU tests, the bench lines, a rocprof of the one-rank FSDP bench
set -o pipefail
T=${TAG:-r4f}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_ddp_gpu.py \
  tests/test_trainer_gpu.py tests/test_model_gpu.py > $O/pytest_dp.log 2>&1 || { tail -30 $O/pytest_dp.log; exit 1; }
tail -2 $O/pytest_dp.log
TAG=$T bash tools/gpu_r4_bench.sh || exit $?
timeout -k 10 300 env GPT2MI_FORCE_COLLECTIVES=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29591 \
  rocprofv3 --kernel-trace --stats -d $O/prof_fsdp -o run -- python bench.py --steps 5 --warmup 3 --no-cpu-baseline \
  --parallel fsdp > $O/prof_fsdp.log 2>&1 || exit $?
python tools/rocpd_stats.py $O/prof_fsdp/run_results.db $O/kernel_stats_fsdp.csv && \
  python tools/prof_summary.py $O/kernel_stats_fsdp.csv 8 > $O/summary_fsdp.txt 2>&1; cat $O/summary_fsdp.txt
