#!/bin/bash
# Round 5 pricing probes: the in-kernel split-K fix-up's tail (tools/fixup_probe.hip, prebuilt into tools/ab/) and the
# attention block map (ATTN_MAP=2: a head's blocks of one half back to back on one XCD) -> gpurun_out/$TAG/
set -o pipefail
O=gpurun_out/${TAG:-r5h}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 tools/ab/fixup_probe > $O/fixup_probe.log 2>&1
rc=$?; cat $O/fixup_probe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 env LIB_AB_OP=attn python tools/lib_ab.py tools/ab/lib_base.so tools/ab/lib_map2.so \
  tools/ab/lib_base.so tools/ab/lib_map2.so > $O/attn_map.log 2>&1
rc=$?; tail -5 $O/attn_map.log; [ $rc -eq 0 ] || exit $rc
