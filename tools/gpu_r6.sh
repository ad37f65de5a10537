#!/bin/bash
# Round 6 GPU step: same-process A/B specs first (tools/lib_ab.py; each spec "name|OP|IMPLS|lib,lib,..."), then an
# optional pytest selection (PYTEST="-k expr" or a file list) -> gpurun_out/$TAG/
set -o pipefail
O=gpurun_out/${TAG:-r6a}
mkdir -p $O
export TMPDIR=/tmp
for spec in "$@"; do
  IFS='|' read -r name op impls libs <<< "$spec"
  timeout -k 10 400 env LIB_AB_OP=$op LIB_AB_IMPLS=$impls python tools/lib_ab.py ${libs//,/ } > $O/$name.log 2>&1
  rc=$?; echo "== $name rc=$rc"; tail -14 $O/$name.log
  [ $rc -eq 0 ] || exit $rc
done
if [ -n "$PYTEST" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu $PYTEST \
    > $O/pytest.log 2>&1
  rc=$?; echo "== pytest rc=$rc"; tail -5 $O/pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python bench.py > $O/bench.log 2>&1; rc=$?
  grep '^{' $O/bench.log | tail -1 > $O/bench.json; echo "bench rc=$rc $(cut -c1-300 $O/bench.json)"
  [ $rc -eq 0 ] || exit $rc
fi
