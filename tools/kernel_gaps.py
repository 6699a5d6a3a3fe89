#!/usr/bin/env python3
"""Idle time between consecutive kernels of a rocprofv3 --kernel-trace run
(rocpd database), by (previous kernel -> next kernel) pair; the window from
the first kernel after a push to the next field kernel (k_efield: the solve
and what precedes it), its kernel time and its gaps; and whole steps (from a
push of the first species to the next one), their span and idle time.

    python tools/kernel_gaps.py <prof_dir> [top]
"""
import glob
import re
import sqlite3
import sys
from collections import defaultdict


def short(name: str) -> str:
    n = re.sub(r"^void ", "", name).replace("(anonymous namespace)::", "")
    n = n.split("(")[0]
    return n[:48]


def main():
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rows = []
    for d in glob.glob(f"{sys.argv[1]}/**/*.db", recursive=True):
        c = sqlite3.connect(d)
        rows += c.execute("select name, start, end from kernels").fetchall()
    rows.sort(key=lambda r: r[1])
    pairs = defaultdict(lambda: [0, 0.0])
    windows = []  # (kernel ns, gap ns, kernels)
    starts = []  # row index of each solve window's first kernel
    gaps = [0] * len(rows)
    inWin = False
    for i in range(1, len(rows)):
        (pn, ps, pe), (nn, ns, ne) = rows[i - 1], rows[i]
        gap = max(0, ns - pe)
        gaps[i] = gap
        if gap < 5e6:  # host-side setup and reporting aside
            p = pairs[(short(pn), short(nn))]
            p[0] += 1
            p[1] += gap
        if short(pn).startswith("k_push") and not short(nn).startswith("k_push"):
            inWin = True
            windows.append([0, 0, 0])
            starts.append(i)
        if inWin:
            w = windows[-1]
            w[0] += ne - ns
            w[1] += gap
            w[2] += 1
            if short(nn).startswith("k_efield"):
                inWin = False
    tot = sum(p[1] for p in pairs.values())
    print(f"kernels {len(rows)}, idle between kernels (gaps < 5 ms) {tot / 1e6:.2f} ms")
    print(f"{'prev -> next':100s} {'count':>6s} {'mean us':>8s} {'total ms':>9s}")
    for (a, b), (n, g) in sorted(pairs.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{a + ' -> ' + b:100s} {n:6d} {g / n / 1e3:8.1f} {g / 1e6:9.3f}")
    ws = [w for w in windows if w[2] > 3][1:]  # skip the first (warm-up)
    if ws:
        k = sum(w[0] for w in ws) / len(ws) / 1e6
        g = sum(w[1] for w in ws) / len(ws) / 1e6
        n = sum(w[2] for w in ws) / len(ws)
        print(f"solve windows {len(ws)}: kernels {k:.3f} ms + gaps {g:.3f} ms per window ({n:.0f} launches)")
    # a step starts at the first push after a field kernel
    steps, sawField = [], False
    for i, r in enumerate(rows):
        n = short(r[0])
        if n.startswith("k_efield"):
            sawField = True
        elif n.startswith("k_push") and sawField:
            steps.append(i)
            sawField = False
    if len(steps) > 3:
        spans = [(rows[b][1] - rows[a][1]) / 1e6 for a, b in zip(steps[1:], steps[2:])]
        idle = [sum(gaps[a + 1:b + 1]) / 1e6 for a, b in zip(steps[1:], steps[2:])]
        med = sorted(range(len(spans)), key=lambda k: idle[k])[len(spans) // 2]
        print(f"whole steps {len(spans)}: median idle {idle[med]:.3f} ms of a {spans[med]:.3f} ms step "
              f"(mean {sum(idle) / len(idle):.3f} of {sum(spans) / len(spans):.3f} ms, sorts and warm-up included)")


if __name__ == "__main__":
    main()
