#!/bin/bash
# whole-step A/B of a variant library (GPT2MI_LIB) against the tree's, alternating bench runs
set -o pipefail
O=gpurun_out/${TAG:-r4nt}
mkdir -p $O
V=${VARIANT:-tools/ab/lib_narrowt.so}
for rep in 1 2; do
  for lib in gpt_2_distributed_amd/libgpt2mi.so $V; do
    n=$(basename $lib .so)_$rep
    timeout -k 10 200 env GPT2MI_LIB=$lib python bench.py --no-cpu-baseline > $O/$n.log 2>&1 || exit $?
    grep '^{' $O/$n.log | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$n',d['value'],d['ms_per_step'])"
  done
done
