"""Reduce the rocprofv3 FETCH_SIZE / WRITE_SIZE passes of tools/kernel_one.py into profiles/traffic.json
(read by bench.py for roofline.traffic).

    python tools/traffic_reduce.py <pmc_root> <probe> [<probe> ...]

<pmc_root>/<probe>_fetch/run_counter_collection.csv and <probe>_write/... are the two passes.
HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE
tallies 128-B wide reads at 64 B).
"""
import csv
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ALGO = {  # algorithmic bytes per launch (operands read once, outputs written once)
    "lm_head_fwd": 2 * (65536 * 768 + 50432 * 768 + 65536 * 50432),
    "lm_head_dgrad": 2 * (65536 * 50432 + 50432 * 768 + 65536 * 768),
    "lm_head_wgrad": 2 * (65536 * 50432 + 65536 * 768) + 4 * 2 * 50432 * 768,
    "fc1_fwd": 2 * (65536 * 768 + 3072 * 768 + 2 * 65536 * 3072) + 4 * 3072,
    "attn_fwd": 2 * (65536 * 2304 + 65536 * 768) + 4 * 768 * 1024,
    # the weight-gradient family, averaged over one step's 25 launches (the tied lm_head + each block's two grouped
    # pairs since round 6; 49 launches before): dY and X read once (bf16), dW read and written once (fp32, accumulated)
    "wgrad": (12 * sum(2 * 65536 * (m + n) + 8 * m * n for m, n in ((2304, 768), (768, 768), (3072, 768), (768, 3072)))
              + 2 * 65536 * (50432 + 768) + 8 * 50432 * 768) // 25,
}
# kernels whose counters make up one probed launch (the wgrad probe = split-K GEMM + slab reduction)
KERNEL_KEY = {"attn_fwd": ("attn_fwd",), "lm_head_wgrad": ("gemm_pp", "splitk_reduce", "transpose_bf16"),
              "wgrad": ("gemm_pp", "splitk_reduce")}  # (the lm_head's one lnf transpose per 25 launches: 0.7 %)
# launches of one repetition of a family probe (the per-launch figure averages the last repetition's launches)
FAMILY = {"wgrad": 25}


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0]


def per_launch(path, counter, keys, family=0):
    total, names = 0.0, []
    for key in keys:
        vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
                if r["Counter_Name"] == counter and key in r["Kernel_Name"]]
        if family:  # a family probe: the mean over its last repetition's launches
            vals = vals[-family:]
        else:
            vals = vals[1:] if len(vals) > 1 else vals  # drop the cold first launch
        total += sum(vals) / len(vals)
        names += sorted({short(r["Kernel_Name"]) for r in csv.DictReader(open(path)) if key in r["Kernel_Name"]})
    return total, " + ".join(names)


def main(root, probes):
    out_path = os.path.join(REPO, "profiles", "traffic.json")
    out = json.load(open(out_path)) if os.path.exists(out_path) else {}
    for p in probes:
        key = KERNEL_KEY.get(p, ("gemm_pp",))
        fam = FAMILY.get(p, 0)
        fetch, kname = per_launch(os.path.join(root, f"{p}_fetch", "run_counter_collection.csv"), "FETCH_SIZE", key,
                                  fam)
        write, _ = per_launch(os.path.join(root, f"{p}_write", "run_counter_collection.csv"), "WRITE_SIZE", key, fam)
        hbm = (2 * fetch + write) * 1024
        out[p] = {"kernel": kname, "fetch_size_kb": round(fetch, 1), "write_size_kb": round(write, 1),
                  "hbm_bytes_per_launch": int(hbm), "algorithmic_bytes_per_launch": ALGO[p],
                  "traffic_over_algorithmic": round(hbm / ALGO[p], 3),
                  "source": f"tools/kernel_one.py {p} under rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate runs)",
                  "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE counts wide reads at 1/2)"}
        print(p, out[p])
    json.dump(out, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
