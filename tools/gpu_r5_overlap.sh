#!/bin/bash
# Round 5: CU-masked streams — where a mask's workgroups run (tools/cumask_probe.hip), then the lm_head forward GEMM
# and the xent pass on disjoint CU sets (tools/overlap_probe.py) -> gpurun_out/$TAG/
set -o pipefail
O=gpurun_out/${TAG:-r5o}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 tools/ab/cumask_probe > $O/cumask_probe.log 2>&1
rc=$?; cat $O/cumask_probe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/overlap_probe.py tools/ab/lib_base.so tools/ab/lib_grid208.so tools/ab/lib_grid224.so \
  > $O/overlap_probe.log 2>&1
rc=$?; cat $O/overlap_probe.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
