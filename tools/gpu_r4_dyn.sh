#!/bin/bash
# The work-queue persistent GEMM (GPT2MI_SCHED_SHARED_CUS): its tests, a same-process A/B against the static walk, and
# the one-rank FSDP / DDP bench lines (which take it while a collective is in flight) beside the plain bench
set -o pipefail
T=${TAG:-r4g}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
git_head=$(cat .git_head 2>/dev/null || echo unknown); echo "$git_head" > $O/TREE
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  -k "persistent_schedule or work_queue" > $O/pytest_dyn.log 2>&1 || { tail -30 $O/pytest_dyn.log; exit 1; }
tail -2 $O/pytest_dyn.log
timeout -k 10 400 env LIB_AB_OP=gemm LIB_AB_IMPLS=0,1024 python tools/lib_ab.py gpt_2_distributed_amd/libgpt2mi.so \
  gpt_2_distributed_amd/libgpt2mi.so > $O/dyn_ab.log 2>&1 || exit $?
tail -12 $O/dyn_ab.log
TAG=$T bash tools/gpu_r4_bench.sh || exit $?
