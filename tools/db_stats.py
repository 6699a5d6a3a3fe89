#!/usr/bin/env python3
"""Kernel statistics (calls, total/avg ns, share) of a rocprofv3 --kernel-trace
--stats output directory (rocpd database) as CSV.

    python tools/db_stats.py <prof_dir> <out.csv>
"""
import glob
import sqlite3
import sys

dbs = glob.glob(f"{sys.argv[1]}/**/*.db", recursive=True)
rows = {}
for d in dbs:
    c = sqlite3.connect(d)
    for name, calls, total, avg, pct in c.execute("select * from top_kernels"):
        r = rows.setdefault(name, [0, 0.0])
        r[0] += calls
        r[1] += total
tot = sum(r[1] for r in rows.values()) or 1.0
with open(sys.argv[2], "w") as f:
    f.write("Name,Calls,TotalDurationNs,AverageNs,Percentage\n")
    for name, (calls, total) in sorted(rows.items(), key=lambda kv: -kv[1][1]):
        f.write('"%s",%d,%.0f,%.1f,%.2f\n' % (name, calls, total * 1e3, total * 1e3 / max(calls, 1), 100 * total / tot))
