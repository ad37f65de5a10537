"""Print the per-launch averages (cold first launch dropped) of rocprofv3 --pmc csvs, per kernel.
    python tools/pmc_show.py <dir-with-run_counter_collection.csv> [...] [--kernel substr]"""
import collections
import csv
import glob
import os
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
sub = next((a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--kernel=")), "")
agg = collections.defaultdict(list)
for d in args:
    for f in glob.glob(os.path.join(d, "**", "run_counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if sub in r["Kernel_Name"]:
                agg[(r["Kernel_Name"].replace("(anonymous namespace)::", "")[:48], r["Counter_Name"])].append(
                    float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    v = v[1:] if len(v) > 1 else v
    print(f"{k:48s} {c:28s} {sum(v) / len(v):.4g}")
