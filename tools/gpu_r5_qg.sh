#!/bin/bash
# Round 5: attention forward with 64 queries per wave (ATTN_FWD_QG=4, 2 waves per workgroup, 2 waves / SIMD) against the
# product form (32 per wave, 4 waves, 3 / SIMD); lib_old = the tree before the QG template (bitwise reference)
set -o pipefail
O=gpurun_out/${TAG:-r5n}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 env LIB_AB_OP=attn python tools/lib_ab.py tools/ab/lib_old.so tools/ab/lib_base.so \
  tools/ab/lib_qg4.so tools/ab/lib_old.so tools/ab/lib_qg4.so > $O/attn_qg.log 2>&1
rc=$?; tail -8 $O/attn_qg.log; [ $rc -eq 0 ] || exit $rc
