set -o pipefail
mkdir -p gpurun_out/exp4
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/exp4/t_gemm.log 2>&1 || { tail -30 gpurun_out/exp4/t_gemm.log; exit 1; }
tail -2 gpurun_out/exp4/t_gemm.log
timeout -k 10 200 python tools/lib_ab.py tools/ab/lib_b0old.so tools/ab/lib_mixed.so > gpurun_out/exp4/wgrad.log 2>&1 || exit $?
cat gpurun_out/exp4/wgrad.log
LIB_AB_OP=gemm timeout -k 10 400 python tools/lib_ab.py tools/ab/lib_b0old.so tools/ab/lib_mixed.so > gpurun_out/exp4/gemm.log 2>&1 || exit $?
cat gpurun_out/exp4/gemm.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/exp4/bench.log 2>&1 || exit $?
tail -1 gpurun_out/exp4/bench.log | cut -c1-300
