#!/usr/bin/env python3
"""Kernel statistics (the `--stats` kernel summary) from a rocprofv3 rocpd database, written as CSV:
Name,Calls,TotalDurationNs,AverageNs,Percentage.  Usage: python scripts/rocpd_stats.py <results.db> <out.csv>"""
import csv
import sqlite3
import sys

con = sqlite3.connect(sys.argv[1])
rows = con.execute("select name, total_calls, total_duration, average, percentage from top_kernels "
                   "order by total_duration desc").fetchall()
unit = con.execute("select avg(duration) from kernels").fetchone()
with open(sys.argv[2], "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "Percentage"])
    for r in rows:
        w.writerow(r)
print(f"{len(rows)} kernels -> {sys.argv[2]}")
