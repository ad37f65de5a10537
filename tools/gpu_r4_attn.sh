#!/bin/bash
# Attention: determinism of the backward, the attention GPU tests, and a same-process A/B of libraries given as
# arguments (first = the tree's library)
set -o pipefail
O=gpurun_out/${TAG:-r4n}
mkdir -p $O
timeout -k 10 200 python tools/attn_determinism.py 12 > $O/determinism.log 2>&1 || { cat $O/determinism.log; exit 1; }
cat $O/determinism.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  -k attention > $O/pytest_attn.log 2>&1 || { tail -30 $O/pytest_attn.log; exit 1; }
tail -1 $O/pytest_attn.log
timeout -k 10 300 env LIB_AB_OP=attn python tools/lib_ab.py "$@" > $O/attn_ab.log 2>&1 || exit $?
grep -v amdgpu.ids $O/attn_ab.log
