#!/bin/bash
# Round 5: the GELU_BWD persistent epilogue with its GELU-derivative operand loaded ahead (PP_AUX_AHEAD 1 / 2) against
# the product (loaded at the start of each 64-row pass) -> gpurun_out/$TAG/
set -o pipefail
O=gpurun_out/${TAG:-r5q}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 env LIB_AB_OP=gemm GEMM_AB_SHAPES=fc2dg,fc1 python tools/lib_ab.py tools/ab/lib_base.so \
  tools/ab/lib_aux1.so tools/ab/lib_aux2.so tools/ab/lib_base.so > $O/aux_ab.log 2>&1
rc=$?; grep -v amdgpu.ids $O/aux_ab.log | tail -8; [ $rc -eq 0 ] || exit $rc
