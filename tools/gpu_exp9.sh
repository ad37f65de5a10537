set -o pipefail
mkdir -p gpurun_out/exp9
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp32_kernels_gpu.py -x -q -m gpu -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/exp9/t_gemm.log 2>&1 || { tail -30 gpurun_out/exp9/t_gemm.log; exit 1; }
tail -2 gpurun_out/exp9/t_gemm.log
LIB_AB_OP=gemm timeout -k 10 400 python tools/lib_ab.py tools/ab/lib_b0old.so tools/ab/lib_cur.so tools/ab/lib_fixdesc.so > gpurun_out/exp9/gemm.log 2>&1 || exit $?
cat gpurun_out/exp9/gemm.log
timeout -k 10 200 python tools/lib_ab.py tools/ab/lib_b0old.so tools/ab/lib_cur.so tools/ab/lib_fixdesc.so > gpurun_out/exp9/wgrad.log 2>&1 || exit $?
cat gpurun_out/exp9/wgrad.log
