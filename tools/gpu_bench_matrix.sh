#!/bin/bash
# The bench lines of one tree: the driver's 1-GPU line, the collective-wrapped step on one forced-RCCL rank (DDP /
# FSDP), GPT-2 350M and 1.5B (the 1.5B FSDP step at BASELINE cfg 5's B=32 with gradient accumulation), and a
# rocprofv3 --kernel-trace --stats profile of the default bench. Outputs under gpurun_out/$TAG/.
set -o pipefail
T=${TAG:-r3b}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
run() {  # name, timeout, command...
  local n=$1 to=$2; shift 2
  echo "== $n"
  timeout -k 10 $to "$@" > $O/$n.log 2>&1
  local rc=$?
  tail -1 $O/$n.log | cut -c1-300
  return $rc
}
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29571"
run bench 300 python bench.py --no-cpu-baseline || exit $?
run ddp1 300 env GPT2MI_FORCE_COLLECTIVES=1 $TR bench.py --gpus 1 --parallel ddp --no-cpu-baseline || exit $?
run fsdp1 300 env GPT2MI_FORCE_COLLECTIVES=1 $TR bench.py --gpus 1 --parallel fsdp --no-cpu-baseline || exit $?
run m350 300 python bench.py --model 350M --batch 32 --steps 10 --warmup 3 --no-cpu-baseline || exit $?
run m15b8 300 python bench.py --model 1.5B --batch 8 --steps 5 --warmup 2 --no-cpu-baseline || exit $?
run m15b_fsdp 600 env GPT2MI_FORCE_COLLECTIVES=1 $TR bench.py --gpus 1 --model 1.5B --batch 32 --grad_accum 2 \
    --steps 3 --warmup 1 --parallel fsdp --no-cpu-baseline || exit $?
echo "== rocprof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --steps 5 --warmup 3 \
    --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
python tools/prof_summary.py $(find $O/prof -name "*kernel_stats.csv" | head -1) 8 > $O/summary.txt 2>&1; head -30 $O/summary.txt
