set -o pipefail
mkdir -p gpurun_out/exp13
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "wgrad" --timeout 200 --timeout-method thread > gpurun_out/exp13/t.log 2>&1 || { tail -30 gpurun_out/exp13/t.log; exit 1; }
tail -2 gpurun_out/exp13/t.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/exp13/prof -o run -- python tools/kernel_one.py lm_head_wgrad_kt 3 > gpurun_out/exp13/prof.log 2>&1 || exit $?
echo ok
