#!/bin/bash
# Same-process A/B runs (tools/lib_ab.py) -> gpurun_out/$TAG/<name>.log; each spec "name|OP|IMPLS|lib,lib,..."
set -o pipefail
O=gpurun_out/${TAG:-r4ab}
mkdir -p $O
export TMPDIR=/tmp
for spec in "$@"; do
  IFS='|' read -r name op impls libs <<< "$spec"
  timeout -k 10 400 env LIB_AB_OP=$op LIB_AB_IMPLS=$impls python tools/lib_ab.py ${libs//,/ } > $O/$name.log 2>&1
  rc=$?; echo "== $name rc=$rc"; tail -12 $O/$name.log
  [ $rc -eq 0 ] || exit $rc
done
