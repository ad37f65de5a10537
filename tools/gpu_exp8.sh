set -o pipefail
mkdir -p gpurun_out/exp8
LIB_AB_OP=gemm LIB_AB_IMPLS=0,9 timeout -k 10 400 python tools/lib_ab.py tools/ab/lib_cur.so tools/ab/lib_cur.so > gpurun_out/exp8/2wg.log 2>&1 || exit $?
cat gpurun_out/exp8/2wg.log
