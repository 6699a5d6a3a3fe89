#!/usr/bin/env python3
"""Per-kernel duration summary of a rocprofv3 --kernel-trace run (rocpd
sqlite output): total / count / mean per kernel name, and the sequence of
k_push dispatches (the template arguments tell sorted from unsorted pushes).

usage: tools/trace_summary.py <rocprofv3 output dir> [top]
"""
import collections
import sqlite3
import sys
from pathlib import Path


def main() -> int:
    d = Path(sys.argv[1])
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 14
    dbs = sorted(d.rglob("*.db"))
    if not dbs:
        print(f"no rocpd database under {d}", file=sys.stderr)
        return 1
    rows = []
    for db in dbs:
        with sqlite3.connect(db) as c:
            rows += list(c.execute("select name, duration from kernels order by start"))
    agg = collections.defaultdict(list)
    for n, dur in rows:
        agg[n[:70]].append(dur / 1e6)
    for n, v in sorted(agg.items(), key=lambda x: -sum(x[1]))[:top]:
        print(f"{sum(v):9.1f} ms {len(v):6d} x {sum(v) / len(v):8.3f} ms  {n}")
    push = [(n.split("(")[0].replace("void ", "").replace("k_push", ""), round(dur / 1e6, 1))
            for n, dur in rows if "k_push" in n]
    print("push sequence:", push)
    return 0


if __name__ == "__main__":
    sys.exit(main())
