#!/bin/bash
# the larger BASELINE models on the final tree: 350M and 1.5B single-process, 1.5B through FSDP at cfg 5's B=32 x 2
set -o pipefail
O=gpurun_out/${TAG:-r4mod}
mkdir -p $O
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29571"
run() {
  local n=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$n.log 2>&1
  local rc=$?
  grep '^{' $O/$n.log | tail -1 > $O/$n.json
  echo "$n rc=$rc $(cut -c1-160 $O/$n.json)"
  return $rc
}
run m350 300 python bench.py --model 350M --batch 32 --steps 10 --warmup 3 --no-cpu-baseline || exit $?
run m15b8 300 python bench.py --model 1.5B --batch 8 --steps 5 --warmup 2 --no-cpu-baseline || exit $?
run m15b_fsdp 600 env GPT2MI_FORCE_COLLECTIVES=1 $TR bench.py --gpus 1 --model 1.5B --batch 32 --grad_accum 2 \
    --steps 3 --warmup 1 --parallel fsdp --no-cpu-baseline || exit $?
