#!/usr/bin/env python3
"""Per-kernel stats (calls, total/avg/min/max ns) from a rocprofv3 rocpd
SQLite database (rocprofv3's default output on ROCm 7), written in the
column layout of rocprofv3's --stats kernel_stats.csv.

    python3 tools/rocpd_stats.py gpurun_out/<tag>/prof/run_results.db > profiles/<name>.csv
"""
import csv
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
rows = db.execute("select name, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
                  "from kernels group by name order by sum(end-start) desc").fetchall()
tot = sum(r[2] for r in rows) or 1
w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
for n, c, t, a, mn, mx in rows:
    w.writerow([n, c, t, round(a, 1), round(100.0 * t / tot, 2), mn, mx])
