set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/exp14
LIB_AB_OP=gemm GEMM_AB_SHAPES="qkv fwd,lm_head fwd" timeout -k 10 300 python tools/lib_ab.py tools/ab/lib_cur.so tools/ab/lib_sc1.so tools/ab/lib_cur.so tools/ab/lib_sc1.so > gpurun_out/exp14/ab.log 2>&1 || exit $?
cat gpurun_out/exp14/ab.log
for v in cur sc1; do
  GPT2MI_LIB=tools/ab/lib_$v.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/exp14/f_$v -o run --output-format csv -- python tools/kernel_one.py lm_head_fwd 3 > gpurun_out/exp14/f_$v.log 2>&1 || exit $?
done
echo pmc ok
