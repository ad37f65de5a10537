#!/bin/bash
# transposed-shadow refresh: its tests, then a kernel-trace profile of the bench (transpose kernel times)
set -o pipefail
O=gpurun_out/${TAG:-r4tr}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  -k "transpose or wgrad_kt" > $O/pytest_tr.log 2>&1 || { tail -30 $O/pytest_tr.log; exit 1; }
tail -1 $O/pytest_tr.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_model_gpu.py \
  > $O/pytest_model.log 2>&1 || { tail -30 $O/pytest_model.log; exit 1; }
tail -1 $O/pytest_model.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --steps 5 --warmup 3 \
  --no-cpu-baseline --probe-every 1000 > $O/prof.log 2>&1 || exit $?
python tools/rocpd_stats.py $O/prof/run_results.db $O/kernel_stats.csv && \
  python tools/prof_summary.py $O/kernel_stats.csv 8 > $O/summary.txt 2>&1
grep -E "transpose|total" $O/summary.txt
