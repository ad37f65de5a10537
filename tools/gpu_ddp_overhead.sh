# The collective-wrapped step on one forced-RCCL rank (DDP / FSDP) beside the unwrapped bench line, same box
set -o pipefail
O=gpurun_out/${TAG:-ddp_overhead}
mkdir -p $O
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29573"
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
timeout -k 10 300 env GPT2MI_FORCE_COLLECTIVES=1 $TR bench.py --gpus 1 --parallel ddp --no-cpu-baseline > $O/ddp1.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench2.log 2>&1 || exit $?
for n in bench ddp1 bench2; do echo "$n $(tail -1 $O/$n.log | cut -c1-200)"; done
