#!/bin/bash
# Round 4: bench lines (default 124M, DDP / FSDP one forced-RCCL rank, 350M FSDP cfg 4) + a rocprof of the default
# bench -> gpurun_out/$TAG/
set -o pipefail
T=${TAG:-r4b}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
run() {  # name, timeout, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1
  local rc=$?
  grep '^{' $O/$name.log | tail -1 > $O/$name.json
  echo "$name rc=$rc $(cut -c1-220 $O/$name.json)"
  return $rc
}
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29581"
run bench 300 python bench.py || exit $?
run ddp1 300 env GPT2MI_FORCE_COLLECTIVES=1 $TR bench.py --no-cpu-baseline --parallel ddp || exit $?
run fsdp1 300 env GPT2MI_FORCE_COLLECTIVES=1 $TR bench.py --no-cpu-baseline --parallel fsdp || exit $?
run bench_again 300 python bench.py --no-cpu-baseline || exit $?
run m350_fsdp 400 env GPT2MI_FORCE_COLLECTIVES=1 $TR bench.py --no-cpu-baseline --parallel fsdp --model 350M --batch 32 \
  --steps 10 --warmup 3 || exit $?
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --steps 5 --warmup 3 \
    --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
  python tools/rocpd_stats.py $O/prof/run_results.db $O/kernel_stats.csv && \
    python tools/prof_summary.py $O/kernel_stats.csv 8 > $O/summary.txt 2>&1; head -32 $O/summary.txt
fi
