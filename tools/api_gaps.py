#!/usr/bin/env python3
"""Host API calls behind the GPU's idle gaps: for a rocprofv3
--kernel-trace --hip-trace run (rocpd database), every gap of at least
`min_us` between consecutive kernels, grouped by (prev -> next) kernel pair,
with the HIP calls the host made from the end of the previous kernel to the
start of the next one (count and total time per call name over the group).
The schema's tables and views go to stdout first when a query fails.

    python tools/api_gaps.py <prof_dir> [min_us] [top_pairs]
    python tools/api_gaps.py <prof_dir> --step [k]   (the k-th whole step,
        default the middle one: every gap of 3 us or more with its HIP calls)
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


def step_timeline(kern, api, k):
    """a step = from a push of the first species after a field kernel to the next"""
    steps, sawField = [], False
    for i, r in enumerate(kern):
        n = short(r[0])
        if n.startswith("k_efield"):
            sawField = True
        elif n.startswith("k_push") and sawField:
            steps.append(i)
            sawField = False
    if len(steps) < 3:
        print("fewer than 3 steps in the trace")
        return
    k = k if k is not None else len(steps) // 2
    a, b = steps[k], steps[k + 1]
    starts = [x[1] for x in api]
    t0 = kern[a][1]
    idle = 0
    print(f"step {k} of {len(steps) - 1}: {(kern[b][1] - t0) / 1e6:.3f} ms, kernels {b - a}")
    for i in range(a + 1, b + 1):
        (pn, ps, pe), (nn, ns, ne) = kern[i - 1], kern[i]
        gap = ns - pe
        if gap <= 0:
            continue
        idle += gap
        if gap < 3e3:
            continue
        j = bisect_left(starts, pe)
        calls = defaultdict(lambda: [0, 0.0])
        while j < len(api) and api[j][1] < ns:
            calls[api[j][0]][0] += 1
            calls[api[j][0]][1] += api[j][2] - api[j][1]
            j += 1
        cs = ", ".join(f"{n.replace('hip', '')}x{c}:{t / 1e3:.0f}" for n, (c, t) in
                       sorted(calls.items(), key=lambda kv: -kv[1][1])[:5])
        print(f"  {(pe - t0) / 1e3:9.1f} us  gap {gap / 1e3:6.1f}  {short(pn)[:30]:30s} -> {short(nn)[:30]:30s} {cs}")
    print(f"idle {idle / 1e3:.1f} us")


def main():
    if len(sys.argv) > 2 and sys.argv[2] == "--step":
        kern, api = [], []
        for d in glob.glob(f"{sys.argv[1]}/**/*.db", recursive=True):
            c = sqlite3.connect(d)
            kern += c.execute("select name, start, end from kernels").fetchall()
            api += c.execute("select name, start, end from regions").fetchall()
        kern.sort(key=lambda r: r[1])
        api.sort(key=lambda r: r[1])
        step_timeline(kern, api, int(sys.argv[3]) if len(sys.argv) > 3 else None)
        return
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
