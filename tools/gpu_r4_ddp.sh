#!/bin/bash
# DDP / FSDP wrappers: the multi-rank GPU tests (goldens, overlap_optimizer variants), the AdamW kernel tests, and the
# one-rank forced-RCCL bench lines beside the plain one
set -o pipefail
T=${TAG:-r4y}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
git_head=$(cat .git_head 2>/dev/null || echo unknown); echo "$git_head" > $O/TREE
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_ddp_gpu.py \
  > $O/pytest_ddp.log 2>&1 || { tail -40 $O/pytest_ddp.log; exit 1; }
tail -2 $O/pytest_ddp.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  -k "adamw or norm" > $O/pytest_adamw.log 2>&1 || { tail -30 $O/pytest_adamw.log; exit 1; }
tail -1 $O/pytest_adamw.log
TAG=$T bash tools/gpu_r4_bench.sh
