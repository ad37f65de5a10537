#!/bin/bash
# Prices attention kernels that read precomputed dropout mask bits: the current library against a probe build whose
# keep masks come from bit extracts (wrong masks, timing only), at p = 0.1, and the current library at p = 0
set -o pipefail
O=gpurun_out/${TAG:-r4h}
mkdir -p $O
timeout -k 10 300 env LIB_AB_OP=attn python tools/lib_ab.py tools/ab/lib_cur.so tools/ab/lib_maskprobe.so \
  > $O/attn_maskprobe.log 2>&1 || exit $?
cat $O/attn_maskprobe.log
timeout -k 10 300 env LIB_AB_OP=attn LIB_AB_PDROP=0 python tools/lib_ab.py tools/ab/lib_cur.so > $O/attn_p0.log 2>&1 || exit $?
cat $O/attn_p0.log
