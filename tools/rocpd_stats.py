#!/usr/bin/env python3
"""Kernel statistics CSV (the `rocprofv3 --stats` kernel_stats layout) from a rocprofv3 run
database (`-d DIR -o run` writes DIR/run_results.db when the output format is rocpd).

usage: python tools/rocpd_stats.py gpurun_out/prof3/run_results.db > profiles/rNN_kernel_stats.csv
"""
import csv
import sqlite3
import sys


def main(path: str) -> None:
    con = sqlite3.connect(path)
    rows = con.execute(
        "select name, count(*), sum(end - start), avg(end - start), min(end - start), max(end - start) "
        "from kernels group by name order by sum(end - start) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_ALL)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, n, tot, avg, mn, mx in rows:
        w.writerow([name, n, tot, f"{avg:.3f}", f"{100.0 * tot / total:.2f}", mn, mx])


if __name__ == "__main__":
    main(sys.argv[1])
