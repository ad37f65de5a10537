# wide (16-B) bf16 slab stores on half-tile map 2 vs map 3: kernel tests, wgrad A/B, step A/B of the new default
set -o pipefail
O=gpurun_out/exp18
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "wgrad or slab" > $O/pytest_wgrad.log 2>&1; rc=$?; tail -2 $O/pytest_wgrad.log; [ $rc -eq 0 ] || exit $rc
LIB_AB_IMPLS=512,512,512,512 timeout -k 10 200 python -u tools/lib_ab.py tools/ab/lib_map3.so \
  gpt_2_distributed_amd/libgpt2mi.so tools/ab/lib_map3.so gpt_2_distributed_amd/libgpt2mi.so \
  > $O/wgrad_map_ab.log 2>&1 || exit $?
cat $O/wgrad_map_ab.log
