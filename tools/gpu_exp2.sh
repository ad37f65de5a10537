set -o pipefail
mkdir -p gpurun_out/exp2
timeout -k 10 120 python tools/trans_ab.py > gpurun_out/exp2/trans_ab.log 2>&1 || exit $?
cat gpurun_out/exp2/trans_ab.log
timeout -k 10 200 python tools/lib_ab.py tools/ab/lib_b0old.so tools/ab/lib_b0new.so > gpurun_out/exp2/wgrad.log 2>&1 || exit $?
cat gpurun_out/exp2/wgrad.log
LIB_AB_OP=gemm timeout -k 10 400 python tools/lib_ab.py tools/ab/lib_b0old.so tools/ab/lib_b0new.so > gpurun_out/exp2/gemm.log 2>&1 || exit $?
cat gpurun_out/exp2/gemm.log
