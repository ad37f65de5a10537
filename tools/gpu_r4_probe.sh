#!/bin/bash
# bench.py's kernel probes: the same bench with every step probed (the round-1..4 behaviour), every 5th (default) and
# only the first step, alternating, to price the event records inside the timed region
set -o pipefail
O=gpurun_out/${TAG:-r4pr}
mkdir -p $O
for rep in 1 2; do
  for pe in 1 5 1000; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --probe-every $pe > $O/bench_pe${pe}_$rep.log 2>&1 || exit $?
    python - $O/bench_pe${pe}_$rep.log $pe <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(f"probe-every {sys.argv[2]:>4}: {d['value']:.0f} tok/s {d['ms_per_step']:.3f} ms  wgrad {d['kernels']['wgrad']['avg_ms']:.4f} ms "
      f"x{d['kernels']['wgrad']['launches']} frac {d['roofline']['frac']}  lm_fwd {d['kernels']['lm_head_fwd']['avg_ms']:.3f}")
PY
  done
done
