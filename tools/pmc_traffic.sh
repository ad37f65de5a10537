#!/bin/bash
# HBM traffic of bench.py's probed kernels: one rocprofv3 --pmc pass per counter (FETCH_SIZE and
# WRITE_SIZE cannot share a pass), over tools/kernel_one.py, reduced into profiles/traffic.json.
# Run on the GPU box from the repo root: bash tools/pmc_traffic.sh
set -e
export TMPDIR=/tmp
OUT=gpurun_out/pmc_traffic
mkdir -p $OUT
for p in ${PROBES:-lm_head_fwd lm_head_dgrad lm_head_wgrad fc1_fwd attn_fwd wgrad}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    d=$OUT/${p}_$( [ $c = FETCH_SIZE ] && echo fetch || echo write )
    timeout -s KILL 120 rocprofv3 --pmc $c -d $d -o run --output-format csv -- python tools/kernel_one.py $p 3 > $d.log 2>&1
  done
done
python tools/traffic_reduce.py $OUT ${PROBES:-lm_head_fwd lm_head_dgrad lm_head_wgrad fc1_fwd attn_fwd wgrad}
