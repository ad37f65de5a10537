set -o pipefail
mkdir -p gpurun_out/exp3
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/exp3/t_gemm.log 2>&1 || { tail -30 gpurun_out/exp3/t_gemm.log; exit 1; }
tail -3 gpurun_out/exp3/t_gemm.log
timeout -k 10 120 python tools/trans_ab.py > gpurun_out/exp3/trans_ab.log 2>&1 || exit $?
cat gpurun_out/exp3/trans_ab.log
timeout -k 10 200 python tools/lib_ab.py tools/ab/lib_b0old.so tools/ab/lib_bufb0old.so tools/ab/lib_b0new.so > gpurun_out/exp3/wgrad.log 2>&1 || exit $?
cat gpurun_out/exp3/wgrad.log
LIB_AB_OP=gemm timeout -k 10 400 python tools/lib_ab.py tools/ab/lib_b0old.so tools/ab/lib_bufb0old.so tools/ab/lib_b0new.so > gpurun_out/exp3/gemm.log 2>&1 || exit $?
cat gpurun_out/exp3/gemm.log
