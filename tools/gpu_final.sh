# Round verification of the committed tree: pytest -m gpu, smoke(), the bench line and a rocprof of the bench -> gpurun_out/$TAG/
set -o pipefail
T=${TAG:-r3d}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --steps 5 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
echo prof ok
