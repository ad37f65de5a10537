#!/bin/bash
# rocprof of the one-rank FSDP / DDP bench lines (forced RCCL collectives) + the GEMM persistent vs non-persistent A/B
set -o pipefail
O=gpurun_out/${TAG:-r4fp}
mkdir -p $O
export TMPDIR=/tmp
for par in fsdp ddp; do
  timeout -k 10 300 env GPT2MI_FORCE_COLLECTIVES=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29591 \
    rocprofv3 --kernel-trace --stats -d $O/prof_$par -o run -- python bench.py --steps 5 --warmup 3 --no-cpu-baseline \
    --parallel $par > $O/prof_$par.log 2>&1 || exit $?
  python tools/rocpd_stats.py $O/prof_$par/run_results.db $O/kernel_stats_$par.csv && \
    python tools/prof_summary.py $O/kernel_stats_$par.csv 8 > $O/summary_$par.txt 2>&1; head -14 $O/summary_$par.txt
done
timeout -k 10 400 env LIB_AB_OP=gemm LIB_AB_IMPLS=0,256 python tools/lib_ab.py gpt_2_distributed_amd/libgpt2mi.so \
  gpt_2_distributed_amd/libgpt2mi.so > $O/persist_ab.log 2>&1 || exit $?
tail -12 $O/persist_ab.log
