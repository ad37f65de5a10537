set -o pipefail
mkdir -p gpurun_out/exp12
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_boundary_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/exp12/t.log 2>&1 || { tail -30 gpurun_out/exp12/t.log; exit 1; }
tail -2 gpurun_out/exp12/t.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/exp12/bench.log 2>&1 || exit $?
tail -1 gpurun_out/exp12/bench.log | cut -c1-300
python - <<'PY'
import json; d = json.loads(open("gpurun_out/exp12/bench.log").read().strip().splitlines()[-1])
print({k: v for k, v in d.get("kernels", {}).items() if "lm_head" in k or k == "wgrad"})
PY
