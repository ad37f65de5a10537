#!/bin/bash
# Work-queue GEMM under CU contention: its tests, then the persistent schedules (static walk, work queue with a static
# first tile = tools/ab/lib_olddyn.so, all-queue = the tree's library, one tile per block) timed alone and beside
# tools/ab/libhog.so holding 32 / 64 CUs; then the one-rank DDP / FSDP bench lines (work queue under collectives)
set -o pipefail
T=${TAG:-r4w}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
git_head=$(cat .git_head 2>/dev/null || echo unknown); echo "$git_head" > $O/TREE
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  -k "persistent_schedule or work_queue" > $O/pytest_dyn.log 2>&1 || { tail -30 $O/pytest_dyn.log; exit 1; }
tail -2 $O/pytest_dyn.log
L=gpt_2_distributed_amd/libgpt2mi.so
for h in 0 32 64; do
  timeout -k 10 400 env LIB_AB_OP=gemm LIB_AB_IMPLS=0,1024,1024,256 LIB_AB_HOG=$h \
    GEMM_AB_SHAPES="qkv fwd,fc1 gelu,fc2dg,proj resid,lm_head fwd" \
    python tools/lib_ab.py $L tools/ab/lib_olddyn.so $L $L > $O/hog$h.log 2>&1 || exit $?
  echo "hog $h"; tail -5 $O/hog$h.log
done
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29581"
for n in ddp fsdp; do
  timeout -k 10 300 env GPT2MI_FORCE_COLLECTIVES=1 $TR bench.py --no-cpu-baseline --parallel $n > $O/$n.log 2>&1 || exit $?
  grep '^{' $O/$n.log | tail -1 | cut -c1-200
done
