set -o pipefail
mkdir -p gpurun_out/exp7
LIB_AB_OP=gemm GEMM_AB_SHAPES="qkv fwd,lm_head fwd,fc1 gelu,proj resid,fc2dg" LIB_AB_STAGGER="0;7000;14000;5000,4;9000,4" timeout -k 10 400 python tools/lib_ab.py tools/ab/lib_cur.so tools/ab/lib_cur.so tools/ab/lib_cur.so tools/ab/lib_cur.so tools/ab/lib_cur.so > gpurun_out/exp7/stagger.log 2>&1 || exit $?
cat gpurun_out/exp7/stagger.log
