#!/usr/bin/env python3
"""Per-dispatch PMC counters of the kernels whose name contains a pattern,
from a rocprofv3 --pmc output directory (rocpd database), as CSV: one row per
dispatch in launch order (the push alternates species within a step).

    python tools/pmc_dispatches.py <prof_dir> <pattern> <out.csv>
"""
import glob
import sqlite3
import sys
from collections import defaultdict


def main():
    d, pat, out = sys.argv[1], sys.argv[2], sys.argv[3]
    rows = defaultdict(dict)
    names = {}
    counters = set()
    for db in glob.glob(f"{d}/**/*.db", recursive=True):
        c = sqlite3.connect(db)
        q = "select dispatch_id, kernel_name, counter_name, value from counters_collection"
        for did, k, cn, v in c.execute(q):
            if pat not in k:
                continue
            rows[did][cn] = rows[did].get(cn, 0.0) + v
            names[did] = k.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
            counters.add(cn)
    cols = sorted(counters)
    with open(out, "w") as f:
        f.write("dispatch,kernel," + ",".join(cols) + "\n")
        for did in sorted(rows):
            f.write(f'{did},"{names[did]}",' + ",".join(f"{rows[did].get(cn, 0):.0f}" for cn in cols) + "\n")
    print(f"{len(rows)} dispatches, counters {cols}")


if __name__ == "__main__":
    main()
