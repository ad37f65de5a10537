#!/bin/bash
# FSDP all-gather fence: the FSDP / DDP GPU tests, then the one-rank FSDP line beside the plain bench (alternating)
set -o pipefail
O=gpurun_out/${TAG:-r4fe}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_ddp_gpu.py \
  > $O/pytest_ddp.log 2>&1 || { tail -40 $O/pytest_ddp.log; exit 1; }
tail -1 $O/pytest_ddp.log
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29581"
for rep in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_$rep.log 2>&1 || exit $?
  timeout -k 10 300 env GPT2MI_FORCE_COLLECTIVES=1 $TR bench.py --no-cpu-baseline --parallel fsdp > $O/fsdp1_$rep.log 2>&1 || exit $?
  for f in bench_$rep fsdp1_$rep; do grep '^{' $O/$f.log | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$f',d['value'],d['ms_per_step'])"; done
done
