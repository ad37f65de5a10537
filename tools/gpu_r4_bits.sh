#!/bin/bash
# Attention keep bits (ABI v12): the attention / model GPU tests, then the attention A/B (hashing vs stored bits, same
# library), the bench lines and a rocprof of the default bench
set -o pipefail
T=${TAG:-r4i}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
git_head=$(cat .git_head 2>/dev/null || echo unknown); echo "$git_head" > $O/TREE
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  -k "attention or fsdp or work_queue" > $O/pytest_attn.log 2>&1 || { tail -30 $O/pytest_attn.log; exit 1; }
tail -2 $O/pytest_attn.log
timeout -k 10 300 env LIB_AB_OP=attn LIB_AB_BITS=0,1 python tools/lib_ab.py tools/ab/lib_bits.so tools/ab/lib_bits.so \
  > $O/attn_bits_ab.log 2>&1 || exit $?
cat $O/attn_bits_ab.log
TAG=$T PROF=1 bash tools/gpu_r4_bench.sh || exit $?
