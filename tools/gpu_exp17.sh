# bf16 split-K slabs: the new kernel tests, the wgrad A/B (fp32 vs bf16 slabs, same library), the whole-step A/B
set -o pipefail
O=gpurun_out/exp17
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "wgrad or slab or pingpong" > $O/pytest_wgrad.log 2>&1; rc=$?; tail -3 $O/pytest_wgrad.log; [ $rc -eq 0 ] || exit $rc
LIB_AB_IMPLS=0,512,0,512 timeout -k 10 200 python -u tools/lib_ab.py gpt_2_distributed_amd/libgpt2mi.so \
  gpt_2_distributed_amd/libgpt2mi.so gpt_2_distributed_amd/libgpt2mi.so gpt_2_distributed_amd/libgpt2mi.so \
  > $O/wgrad_slab16_ab.log 2>&1 || exit $?
cat $O/wgrad_slab16_ab.log
timeout -k 10 300 python -u tools/step_ab.py wgrad_bf16_slabs False True --rounds 4 --steps 10 > $O/step_ab.log 2>&1 || exit $?
cat $O/step_ab.log
