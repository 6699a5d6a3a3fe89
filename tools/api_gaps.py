#!/usr/bin/env python3
"""Host API calls behind the GPU's idle gaps: for a rocprofv3
--kernel-trace --hip-trace run (rocpd database), every gap of at least
`min_us` between consecutive kernels, grouped by (prev -> next) kernel pair,
with the HIP calls the host made from the end of the previous kernel to the
start of the next one (count and total time per call name over the group).
The schema's tables and views go to stdout first when a query fails.

    python tools/api_gaps.py <prof_dir> [min_us] [top_pairs]
"""
import glob
import re
import sqlite3
import sys
from bisect import bisect_left
from collections import defaultdict


def short(name: str) -> str:
    n = re.sub(r"^void ", "", name).replace("(anonymous namespace)::", "")
    return n.split("(")[0][:48]


def main():
    minUs = float(sys.argv[2]) if len(sys.argv) > 2 else 50.0
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    kern, api = [], []
    for d in glob.glob(f"{sys.argv[1]}/**/*.db", recursive=True):
        c = sqlite3.connect(d)
        kern += c.execute("select name, start, end from kernels").fetchall()
        try:
            api += c.execute("select name, start, end from regions").fetchall()
        except sqlite3.Error as e:
            print("regions query failed:", e)
            for t, n in c.execute("select type, name from sqlite_master where type in ('table', 'view')"):
                print(" ", t, n)
            return
    kern.sort(key=lambda r: r[1])
    api.sort(key=lambda r: r[1])
    starts = [a[1] for a in api]
    groups = defaultdict(lambda: {"n": 0, "gap": 0.0, "calls": defaultdict(lambda: [0, 0.0])})
    for (pn, ps, pe), (nn, ns, ne) in zip(kern, kern[1:]):
        gap = ns - pe
        if gap < minUs * 1e3 or gap > 5e6:
            continue
        g = groups[(short(pn), short(nn))]
        g["n"] += 1
        g["gap"] += gap
        i = bisect_left(starts, pe)
        while i < len(api) and api[i][1] < ns:
            name, s, e = api[i]
            cl = g["calls"][name]
            cl[0] += 1
            cl[1] += e - s
            i += 1
    for (a, b), g in sorted(groups.items(), key=lambda kv: -kv[1]["gap"])[:top]:
        print(f"{a} -> {b}: {g['n']} gaps, mean {g['gap'] / g['n'] / 1e3:.1f} us")
        for name, (n, t) in sorted(g["calls"].items(), key=lambda kv: -kv[1][1])[:10]:
            print(f"    {name[:60]:60s} {n / g['n']:6.1f} per gap {t / g['n'] / 1e3:9.1f} us per gap")


if __name__ == "__main__":
    main()
