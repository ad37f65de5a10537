#!/bin/bash
# Round 5: HIP runtime settings A/B on the default bench (alternating runs, one box): HIP_FORCE_DEV_KERNARG -> gpurun_out/$TAG/
set -o pipefail
O=gpurun_out/${TAG:-r5v}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for v in 0 1; do
    timeout -k 10 300 env HIP_FORCE_DEV_KERNARG=$v python bench.py --no-cpu-baseline > $O/bench_k${v}_$r.log 2>&1 || exit $?
    echo "kernarg=$v run $r: $(grep '^{' $O/bench_k${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
