#!/bin/bash
# Round 5: packed vs scalar f32 issue cost (tools/valu_probe2.hip) and the attention A/B of scalar softmax pairs
# (ATTN_PK=0) and the 24-bit closing hash multiply (DROP_MUL24=1, other masks: timing only) -> gpurun_out/$TAG/
set -o pipefail
O=gpurun_out/${TAG:-r5i}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 tools/ab/valu_probe2 > $O/valu_probe2.log 2>&1
rc=$?; cat $O/valu_probe2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 env LIB_AB_OP=attn python tools/lib_ab.py tools/ab/lib_base.so tools/ab/lib_pk0.so \
  tools/ab/lib_m24.so tools/ab/lib_pk0m24.so tools/ab/lib_base.so tools/ab/lib_pk0.so > $O/attn_pk.log 2>&1
rc=$?; tail -8 $O/attn_pk.log; [ $rc -eq 0 ] || exit $rc
