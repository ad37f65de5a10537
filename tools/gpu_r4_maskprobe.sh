#!/bin/bash
# Prices attention kernels that read precomputed dropout mask bits: the current library against a probe build whose
# keep masks come from bit extracts (wrong masks, timing only), at p = 0.1; and per-kernel times (rocprof) of the
# current library at p = 0.1 and p = 0 (what dropout costs each kernel)
set -o pipefail
O=gpurun_out/${TAG:-r4h}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 env LIB_AB_OP=attn python tools/lib_ab.py tools/ab/lib_cur.so tools/ab/lib_maskprobe.so \
  > $O/attn_maskprobe.log 2>&1 || exit $?
cat $O/attn_maskprobe.log
for p in 0.1 0; do
  timeout -k 10 300 env LIB_AB_OP=attn LIB_AB_PDROP=$p rocprofv3 --kernel-trace --stats -d $O/prof_attn_$p -o run -- \
    python tools/lib_ab.py tools/ab/lib_cur.so > $O/attn_p$p.log 2>&1 || exit $?
  python tools/rocpd_stats.py $O/prof_attn_$p/run_results.db $O/attn_stats_$p.csv && \
    python tools/prof_summary.py $O/attn_stats_$p.csv 1 > $O/attn_summary_$p.txt 2>&1; head -5 $O/attn_summary_$p.txt
done
