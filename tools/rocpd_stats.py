"""Kernel statistics (the --stats table) from a rocprofv3 rocpd SQLite database.
usage: python tools/rocpd_stats.py <results.db> [out.csv]"""
import csv
import sqlite3
import sys

db = sys.argv[1]
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name_col = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else None)
rows = c.execute(f"select {name_col}, start, end from kernels").fetchall()
agg = {}
for name, s, e in rows:
    d = agg.setdefault(name, [])
    d.append(e - s)
tot = sum(sum(v) for v in agg.values())
out = []
for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    n = len(v)
    avg = sum(v) / n
    sd = (sum((x - avg) ** 2 for x in v) / max(1, n - 1)) ** 0.5
    out.append([name, n, sum(v), avg, 100.0 * sum(v) / tot, min(v), max(v), sd])
hdr = ["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"]
w = csv.writer(open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
w.writerow(hdr)
for r in out:
    w.writerow(r)
