set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG:-r3a}_t.log 2>&1
rc=$?
tail -5 gpurun_out/${TAG:-r3a}_t.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG:-r3a}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG:-r3a}_bench.log | cut -c1-400
timeout -k 10 300 python bench.py --model 1.5B --batch 8 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG:-r3a}_bench15.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG:-r3a}_bench15.log | cut -c1-600
