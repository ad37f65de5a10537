#!/bin/bash
# kernel trace of the bench step without timing probes: the idle gaps at kernel boundaries
set -o pipefail
O=gpurun_out/${TAG:-r4gap}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run -- python bench.py --steps 5 --warmup 3 \
  --no-cpu-baseline --probe-every 1000 > $O/prof.log 2>&1 || exit $?
ls $O/prof
