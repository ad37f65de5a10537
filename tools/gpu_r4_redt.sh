#!/bin/bash
# transposing split-K reduce: its bitwise tests, and a kernel-trace profile of the default bench (summary + the
# reduce's line)
set -o pipefail
T=${TAG:-r4z}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  -k "wgrad" > $O/pytest_wgrad.log 2>&1 || { tail -30 $O/pytest_wgrad.log; exit 1; }
tail -1 $O/pytest_wgrad.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --steps 5 --warmup 3 \
  --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
python tools/rocpd_stats.py $O/prof/run_results.db $O/kernel_stats.csv && \
  python tools/prof_summary.py $O/kernel_stats.csv 8 > $O/summary.txt 2>&1
grep -E "splitk_reduce|total" $O/summary.txt
