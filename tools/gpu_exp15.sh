set -o pipefail
mkdir -p gpurun_out/exp15
LIB_AB_OP=gemm GEMM_AB_SHAPES="qkv fwd,lm_head fwd,fc1shape bf16" timeout -k 10 300 python tools/lib_ab.py tools/ab/lib_bf16img.so tools/ab/lib_direct.so tools/ab/lib_bf16img.so tools/ab/lib_direct.so > gpurun_out/exp15/ab.log 2>&1 || exit $?
cat gpurun_out/exp15/ab.log
