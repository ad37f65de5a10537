#!/bin/bash
# A/B of the ping-pong GEMM's tile-group height (GPT2MI_PP_GM 4 = the tree, 8, 16, 32): same-process timing of the
# forward / dgrad shapes (tools/lib_ab.py gemm mode) and the lm_head forward's fabric fetch bytes per variant
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab_gm
mkdir -p $O
L=gpt_2_distributed_amd/libgpt2mi.so
LIB_AB_OP=gemm GEMM_AB_SHAPES="lm_head,qkv,fc1 gelu,fc2dg" timeout -k 10 300 python tools/lib_ab.py $L tools/ab/lib_gm8.so \
  tools/ab/lib_gm16.so tools/ab/lib_gm32.so > $O/ab.log 2>&1 || exit $?
cat $O/ab.log
for v in tree gm8 gm16 gm32; do
  lib=$L; [ $v = tree ] || lib=tools/ab/lib_$v.so
  for c in FETCH_SIZE WRITE_SIZE; do
    GPT2MI_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $c -d $O/${v}_$c -o run --output-format csv -- \
      python tools/kernel_one.py lm_head_fwd 3 > $O/${v}_$c.log 2>&1 || exit $?
  done
  python tools/pmc_show.py $O/${v}_FETCH_SIZE $O/${v}_WRITE_SIZE --kernel=gemm_pp | sed "s/^/$v /"
done
