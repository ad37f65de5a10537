# persistent schedule up to K = 4096 by default: the schedule-equivalence tests, the GEMM A/B (auto vs one tile per
# block), the bench line
set -o pipefail
O=gpurun_out/exp19
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k "persistent or pingpong or edge" > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
GEMM_AB_SHAPES="qkv dgrad,fc1 dgrad,fc2 fwd,lm_head dgrad" timeout -k 10 300 python -u tools/gemm_ab.py 0 6 > $O/gemm_ab.log 2>&1 || exit $?
cat $O/gemm_ab.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-250
