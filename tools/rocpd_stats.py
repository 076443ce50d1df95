#!/usr/bin/env python3
"""Kernel stats from a rocprofv3 rocpd database (ROCm 7 default output) as the --stats CSV columns.

usage: rocpd_stats.py <run_results.db> [out.csv]
"""
import csv
import sqlite3
import sys


def main():
    db, out = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else None)
    c = sqlite3.connect(db)
    rows = c.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
        "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    f = open(out, "w", newline="") if out else sys.stdout
    w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, n, tot, avg, mn, mx in rows:
        w.writerow([name, n, int(tot), round(avg, 1), round(100.0 * tot / total, 4), int(mn), int(mx)])
    if out:
        f.close()


if __name__ == "__main__":
    main()
