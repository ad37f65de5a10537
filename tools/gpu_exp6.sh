set -o pipefail
mkdir -p gpurun_out/exp6
LIB_AB_OP=gemm GEMM_AB_SHAPES="qkv fwd,lm_head fwd,fc1 gelu,proj resid,fc2dg,fc1shape bf16" timeout -k 10 300 python tools/lib_ab.py tools/ab/lib_cur.so tools/ab/lib_nostore.so tools/ab/lib_noepi.so > gpurun_out/exp6/epi.log 2>&1 || exit $?
cat gpurun_out/exp6/epi.log
