#!/usr/bin/env python3
"""Per-dispatch durations of the push kernels in a rocprofv3 --kernel-trace
run (rocpd database), in launch order, with the kernel instance:

    python tools/push_dispatches.py <prof_dir>
"""
import glob
import re
import sqlite3
import sys


def main():
    rows = []
    for d in glob.glob(f"{sys.argv[1]}/**/*.db", recursive=True):
        c = sqlite3.connect(d)
        rows += c.execute("select name, start, end from kernels").fetchall()
    rows.sort(key=lambda r: r[1])
    prev = None
    for name, s, e in rows:
        n = re.sub(r"^void ", "", name).replace("(anonymous namespace)::", "").split("(")[0]
        if n.startswith("k_push"):
            gap = (s - prev) / 1e6 if prev else 0.0
            print(f"{n:40s} {(e - s) / 1e6:8.3f} ms  (start {gap:8.3f} ms after the previous push started)")
            prev = s


if __name__ == "__main__":
    main()
