#!/bin/bash
# Round 6: alternating bench runs of the step under two or more settings (SIDES="A B C", env assignments AB_A, AB_B, ...)
# -> gpurun_out/$TAG/ab_{A,B}_{i}.json; optional pytest selection first (PYTEST)
set -o pipefail
O=gpurun_out/${TAG:-r6b}
mkdir -p $O
export TMPDIR=/tmp
if [ -n "$PYTEST" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu $PYTEST \
    > $O/pytest.log 2>&1
  rc=$?; echo "== pytest rc=$rc"; tail -5 $O/pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
for i in $(seq 1 ${ROUNDS:-2}); do
  for side in ${SIDES:-A B}; do
    v=AB_$side; envs="${!v:-X_AB=$side}"
    timeout -k 10 300 env $envs python bench.py --no-cpu-baseline ${BENCH_ARGS} > $O/ab_${side}_$i.log 2>&1; rc=$?
    grep '^{' $O/ab_${side}_$i.log | tail -1 > $O/ab_${side}_$i.json
    echo "$side $i rc=$rc $(python -c "import json;d=json.load(open('$O/ab_${side}_$i.json'));print(d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['achieved'])")"
    [ $rc -eq 0 ] || exit $rc
  done
done
