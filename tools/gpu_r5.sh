#!/bin/bash
# Round 5 GPU step: an optional pytest selection (PYTEST="-k expr" or a file list), then same-process A/B specs
# (tools/lib_ab.py; each spec "name|OP|IMPLS|lib,lib,..." with optional GEMM_AB_SHAPES in the env) -> gpurun_out/$TAG/
set -o pipefail
O=gpurun_out/${TAG:-r5a}
mkdir -p $O
export TMPDIR=/tmp
if [ -n "$PYTEST" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu $PYTEST \
    > $O/pytest.log 2>&1
  rc=$?; echo "== pytest rc=$rc"; tail -5 $O/pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
for spec in "$@"; do
  IFS='|' read -r name op impls libs <<< "$spec"
  timeout -k 10 400 env LIB_AB_OP=$op LIB_AB_IMPLS=$impls python tools/lib_ab.py ${libs//,/ } > $O/$name.log 2>&1
  rc=$?; echo "== $name rc=$rc"; tail -14 $O/$name.log
  [ $rc -eq 0 ] || exit $rc
done
