#!/bin/bash
# PMC passes on the current tree: HBM traffic of bench.py's probed kernels (tools/pmc_traffic.sh -> gpurun_out/pmc_traffic,
# reduced here into profiles/traffic.json) and the SQ issue / wait / MFMA-busy counters of the step's kernel families
# (tools/gpu_sq.sh -> gpurun_out/sq_r4)
set -o pipefail
bash tools/pmc_traffic.sh > gpurun_out/pmc_traffic.log 2>&1 || { tail -20 gpurun_out/pmc_traffic.log; exit 1; }
tail -12 gpurun_out/pmc_traffic.log
OUT=gpurun_out/sq_r4 bash tools/gpu_sq.sh > gpurun_out/sq_r4.log 2>&1 || { tail -20 gpurun_out/sq_r4.log; exit 1; }
cat gpurun_out/sq_r4/summary.txt
