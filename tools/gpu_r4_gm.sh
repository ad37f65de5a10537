#!/bin/bash
# Tile grouping GM of the persistent GEMM (tools/ab/lib_gm{4,8,16}.so): same-process time A/B on the forward shapes,
# then the lm_head forward's FETCH_SIZE / WRITE_SIZE per variant (one --pmc pass each)
set -o pipefail
O=gpurun_out/${TAG:-r4gm}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 env LIB_AB_OP=gemm GEMM_AB_SHAPES="lm_head fwd,qkv fwd,fc1 gelu,proj resid" python tools/lib_ab.py \
  tools/ab/lib_gm4.so tools/ab/lib_gm8.so tools/ab/lib_gm16.so tools/ab/lib_gm4.so > $O/gm_ab.log 2>&1 || exit $?
grep -v amdgpu.ids $O/gm_ab.log
for v in 4 8 16; do
  for c in FETCH_SIZE WRITE_SIZE; do
    d=$O/gm${v}_$c
    timeout -s KILL 120 env GPT2MI_LIB=tools/ab/lib_gm$v.so rocprofv3 --pmc $c -d $d -o run --output-format csv -- \
      python tools/kernel_one.py lm_head_fwd 3 > $d.log 2>&1 || exit $?
  done
done
O=$O python - <<'PY'
import csv, glob, os
O = os.environ.get("O", "gpurun_out/" + os.environ.get("TAG", "r4gm"))
for v in (4, 8, 16):
    tot = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = glob.glob(f"{O}/gm{v}_{c}/**/*counter_collection.csv", recursive=True)
        vals = []
        for row in csv.DictReader(open(f[0])):
            if "gemm_pp_kernel" in row.get("Kernel_Name", "") and row.get("Counter_Name") == c:
                vals.append(float(row["Counter_Value"]))
        tot[c] = sum(vals) / max(1, len(vals))
    gb = (2 * tot["FETCH_SIZE"] + tot["WRITE_SIZE"]) * 1024 / 1e9
    print(f"GM={v}: fetch {tot['FETCH_SIZE']/1e6:.2f} GB(raw KB/1e6) write {tot['WRITE_SIZE']/1e6:.2f}  corrected {gb:.2f} GB per launch")
PY
