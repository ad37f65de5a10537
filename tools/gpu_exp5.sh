set -o pipefail
mkdir -p gpurun_out/exp5
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp32_kernels_gpu.py -x -q -m gpu -k "attn or drop" --timeout 120 --timeout-method thread > gpurun_out/exp5/t_attn.log 2>&1 || { tail -30 gpurun_out/exp5/t_attn.log; exit 1; }
tail -2 gpurun_out/exp5/t_attn.log
LIB_AB_OP=attn timeout -k 10 200 python tools/lib_ab.py tools/ab/lib_attnold.so tools/ab/lib_attnnew.so tools/ab/lib_attnold.so tools/ab/lib_attnnew.so > gpurun_out/exp5/attn.log 2>&1 || exit $?
cat gpurun_out/exp5/attn.log
