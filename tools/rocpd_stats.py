"""Kernel statistics CSV (rocprofv3 --stats layout) from a rocprofv3 rocpd database.

    python tools/rocpd_stats.py <run_results.db> <out.csv>

Columns: Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs, StdDev — per kernel
name over every dispatch in the database (the `kernels` view: start / end in ns)."""
import csv
import sqlite3
import sys

import numpy as np

db, out = sys.argv[1], sys.argv[2]
c = sqlite3.connect(db)
rows = c.execute("select name, \"end\" - start from kernels").fetchall()
by = {}
for name, d in rows:
    by.setdefault(name, []).append(float(d))
tot = sum(sum(v) for v in by.values())
with open(out, "w", newline="") as fh:
    w = csv.writer(fh, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        a = np.array(v)
        w.writerow([name, len(a), a.sum(), a.mean(), 100.0 * a.sum() / tot, a.min(), a.max(), a.std(ddof=1) if len(a) > 1 else 0.0])
