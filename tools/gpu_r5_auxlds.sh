#!/bin/bash
# Round 5: the GELU_BWD epilogue with a bf16 image and LDS-DMA'd derivative rows one pass ahead (PP_AUX_LDS=1): numerics
# (tools/aux_check.py) and same-process timing against the product -> gpurun_out/$TAG/
set -o pipefail
O=gpurun_out/${TAG:-r5r}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/aux_check.py tools/ab/lib_base.so tools/ab/lib_auxlds.so > $O/aux_check.log 2>&1
rc=$?; grep -v amdgpu.ids $O/aux_check.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 env LIB_AB_OP=gemm GEMM_AB_SHAPES=fc2dg,fc1shape\ bf16 python tools/lib_ab.py tools/ab/lib_base.so \
  tools/ab/lib_auxlds.so tools/ab/lib_base.so tools/ab/lib_auxlds.so > $O/auxlds_ab.log 2>&1
rc=$?; grep -v amdgpu.ids $O/auxlds_ab.log | tail -6; [ $rc -eq 0 ] || exit $rc
