#!/bin/bash
# kernel-trace stats of the one-rank FSDP bench (no timing probes)
set -o pipefail
O=gpurun_out/${TAG:-r4fe}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 env GPT2MI_FORCE_COLLECTIVES=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29591 \
  rocprofv3 --kernel-trace --stats -d $O/prof_fsdp -o run -- python bench.py --steps 5 --warmup 3 --no-cpu-baseline \
  --parallel fsdp --probe-every 1000 > $O/prof_fsdp.log 2>&1 || exit $?
python tools/rocpd_stats.py $O/prof_fsdp/run_results.db $O/kernel_stats_fsdp.csv && \
  python tools/prof_summary.py $O/kernel_stats_fsdp.csv 8 > $O/summary_fsdp.txt 2>&1; grep -E "gemm_pp_kernel<false, false|total" $O/summary_fsdp.txt
