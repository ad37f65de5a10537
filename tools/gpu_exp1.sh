set -o pipefail
mkdir -p gpurun_out/exp1
timeout -k 10 120 python tools/trans_ab.py > gpurun_out/exp1/trans_ab.log 2>&1 || exit $?
cat gpurun_out/exp1/trans_ab.log
LIB_AB_OP=gemm GEMM_AB_SHAPES="qkv fwd,lm_head fwd,fc1 gelu,proj resid,fc2dg" timeout -k 10 300 python tools/lib_ab.py tools/ab/lib_base.so tools/ab/lib_nostore.so tools/ab/lib_l2store.so > gpurun_out/exp1/store.log 2>&1 || exit $?
cat gpurun_out/exp1/store.log
timeout -k 10 200 python tools/lib_ab.py tools/ab/lib_base.so tools/ab/lib_nolgkm.so > gpurun_out/exp1/lgkm_wgrad.log 2>&1 || exit $?
cat gpurun_out/exp1/lgkm_wgrad.log
LIB_AB_OP=gemm GEMM_AB_SHAPES="qkv fwd,lm_head,fc1 dgrad,fc1 gelu" timeout -k 10 300 python tools/lib_ab.py tools/ab/lib_base.so tools/ab/lib_nolgkm.so > gpurun_out/exp1/lgkm_gemm.log 2>&1 || exit $?
cat gpurun_out/exp1/lgkm_gemm.log
