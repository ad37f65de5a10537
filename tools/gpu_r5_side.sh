#!/bin/bash
# Side-stream weight gradients (Engine.SIDE_WGRAD): the full-step goldens with the side stream on, then alternating
# bench runs off / on / on + work-queue GEMMs -> gpurun_out/$TAG/
set -o pipefail
O=gpurun_out/${TAG:-r5e}
mkdir -p $O
export TMPDIR=/tmp
GPT2MI_SIDE_WGRAD=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_model_gpu.py > $O/pytest_side.log 2>&1
rc=$?; tail -3 $O/pytest_side.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in "0 0" "1 0" "1 1"; do
    set -- $v
    timeout -k 10 300 env GPT2MI_SIDE_WGRAD=$1 GPT2MI_SIDE_SHARED=$2 python bench.py --no-cpu-baseline \
      > $O/bench_s$1$2_$r.log 2>&1 || exit $?
    echo "side=$1 shared=$2 run $r: $(grep '^{' $O/bench_s$1$2_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
