"""rocprofv3 --kernel-trace database (rocpd SQLite, this ROCm's default output) -> the kernel_stats.csv of
`--output-format csv` (Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs), for
tools/prof_summary.py.

    python tools/rocpd_stats.py <run_results.db> <out kernel_stats.csv>
"""
import csv
import sqlite3
import sys


def main(db, out):
    con = sqlite3.connect(db)
    tables = {r[0].split("_0")[0]: r[0] for r in con.execute("select name from sqlite_master where type='table'")}
    kd, ks = tables["rocpd_kernel_dispatch"], tables["rocpd_info_kernel_symbol"]
    rows = con.execute(f"select s.display_name, count(*), sum(d.end - d.start), min(d.end - d.start), "
                       f"max(d.end - d.start) from {kd} d join {ks} s on d.kernel_id = s.id "
                       f"group by s.display_name").fetchall()
    tot = sum(r[2] for r in rows)
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, n, s, mn, mx in sorted(rows, key=lambda r: -r[2]):
            w.writerow([name, n, s, s / n, 100.0 * s / tot, mn, mx])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
