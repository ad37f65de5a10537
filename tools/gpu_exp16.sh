set -o pipefail
export TMPDIR=/tmp
PROBES="lm_head_fwd lm_head_dgrad lm_head_wgrad fc1_fwd attn_fwd wgrad" timeout -k 10 900 bash tools/pmc_traffic.sh > gpurun_out/pmc_traffic.log 2>&1 || { tail -20 gpurun_out/pmc_traffic.log; exit 1; }
tail -8 gpurun_out/pmc_traffic.log
cp profiles/traffic.json gpurun_out/traffic.json
OUT=gpurun_out/sq_r3g PROBES="wgrad lm_head_fwd attn_bwd" timeout -k 10 600 bash tools/gpu_sq.sh > gpurun_out/sq_r3g.log 2>&1 || { tail -20 gpurun_out/sq_r3g.log; exit 1; }
cat gpurun_out/sq_r3g/summary.txt
