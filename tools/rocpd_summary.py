#!/usr/bin/env python3
"""Write the per-kernel summary (rocprofv3 --stats equivalent) of a rocprofv3
sqlite output (*_results.db) as CSV: name,calls,total_ns,avg_ns,percent."""
import csv
import sqlite3
import sys

db, out = sys.argv[1], sys.argv[2]
c = sqlite3.connect(db)
rows = c.execute("select name,total_calls,total_duration,average,percentage from top_kernels").fetchall()
with open(out, "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
    for r in rows:
        w.writerow(r)
print(open(out).read())
