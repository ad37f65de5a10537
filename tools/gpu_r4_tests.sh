#!/bin/bash
# Round 4: the GPU test suite, smoke() and the slab-precision report on the current tree -> gpurun_out/$TAG/
set -o pipefail
T=${TAG:-r4a}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
git_head=$(cat .git_head 2>/dev/null || echo unknown); echo "$git_head" > $O/TREE
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -s --timeout 100 \
  -k slab_precision_per_element > $O/slab_precision.log 2>&1 || { tail -20 $O/slab_precision.log; exit 1; }
grep "per-element" $O/slab_precision.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
