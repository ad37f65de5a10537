#!/bin/bash
# SQ counters (two rocprofv3 --pmc passes each, tools/pmc_sq.sh) of the step's main kernel families -> $OUT
set -e
OUT=${OUT:-gpurun_out/sq_r3}
mkdir -p $OUT
for p in ${PROBES:-attn_fwd attn_bwd wgrad lm_head_fwd lm_head_dgrad fc1_fwd proj_fwd fc2_dgrad qkv_fwd fc2_fwd}; do
  echo "== $p"
  bash tools/pmc_sq.sh $p $OUT/$p
done
python tools/sq_summary.py $OUT/* > $OUT/summary.txt
cat $OUT/summary.txt
