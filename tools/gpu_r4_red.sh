#!/bin/bash
# split-K reduction variants: the wgrad family probe under rocprof with each library, per-kernel averages
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4v
mkdir -p $O
cp gpt_2_distributed_amd/libgpt2mi.so /tmp/lib_keep.so
for v in cur red1 red2; do
  cp tools/ab/lib_$v.so gpt_2_distributed_amd/libgpt2mi.so
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python tools/kernel_one.py wgrad 5 \
    > $O/prof_$v.log 2>&1 || { cp /tmp/lib_keep.so gpt_2_distributed_amd/libgpt2mi.so; exit 1; }
  python tools/rocpd_stats.py $O/prof_$v/run_results.db $O/stats_$v.csv && grep -i "reduce\|gemm_pp" $O/stats_$v.csv | cut -c1-160
done
cp /tmp/lib_keep.so gpt_2_distributed_amd/libgpt2mi.so
