#!/usr/bin/env python3
"""Kernel statistics CSV (the rocprofv3 --stats columns) from a rocprofv3
rocpd database (run_results.db), for runs recorded without
--output-format csv.  Durations in ns, as rocprofv3's kernel_stats.csv.
usage: rocpd_stats.py <run_results.db> <out.csv>
"""
import csv
import sqlite3
import sys


def main():
    db, out = sys.argv[1], sys.argv[2]
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    with open(out, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, n, tot, avg, mn, mx in rows:
            w.writerow([name, n, tot, round(avg, 1), round(100.0 * tot / total, 4), mn, mx])
    print(open(out).read())


if __name__ == "__main__":
    main()
