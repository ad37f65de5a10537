set -o pipefail
mkdir -p gpurun_out/exp10
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/exp10/t_gemm.log 2>&1 || { tail -30 gpurun_out/exp10/t_gemm.log; exit 1; }
tail -2 gpurun_out/exp10/t_gemm.log
LIB_AB_OP=gemm GEMM_AB_SHAPES="qkv fwd,lm_head fwd,fc1shape bf16" timeout -k 10 400 python tools/lib_ab.py tools/ab/lib_cur.so tools/ab/lib_bf16img.so tools/ab/lib_cur.so tools/ab/lib_bf16img.so > gpurun_out/exp10/gemm.log 2>&1 || exit $?
cat gpurun_out/exp10/gemm.log
