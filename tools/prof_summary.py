"""Summarise a rocprofv3 --kernel-trace --stats run of bench.py: ms per step per kernel.

    python tools/prof_summary.py <run_kernel_stats.csv> <profiled steps>
"""
import csv
import sys


def main(path, steps):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        ms = float(r["TotalDurationNs"]) / steps / 1e6
        if ms < 0.02:
            continue
        print(f'{ms:7.2f} ms/step {int(r["Calls"]) / steps:6.1f}/step {float(r["AverageNs"]) / 1e3:9.1f} us  '
              f'{r["Name"][:90]}')
    print(f"total GPU time {tot / steps / 1e6:.2f} ms/step")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
