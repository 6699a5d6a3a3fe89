#!/usr/bin/env python3
"""Mean value per dispatch of every counter in a rocprofv3 --pmc output
directory, for the kernels with a grid of at least 2^20 work-items.

    python tools/pmc_kernels.py <pmc_dir> [out.json]
"""
import json
import os
import sqlite3
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_summary import short  # noqa: E402


def main() -> int:
    d = Path(sys.argv[1])
    dbs = list(d.rglob("*.db"))
    per = defaultdict(lambda: defaultdict(list))
    for db in dbs:
        c = sqlite3.connect(db)
        q = "select kernel_name, grid_size, counter_name, value from counters_collection"
        for k, g, n, v in c.execute(q):
            if int(g) >= int(os.environ.get("PMC_MIN_GRID", 1 << 20)):
                per[(short(k), int(g))][n].append(float(v))
    out = {f"{k[0]} grid={k[1]}": {n: {"mean": sum(v) / len(v), "n": len(v)} for n, v in cs.items()}
           for k, cs in per.items()}
    text = json.dumps(out, indent=1)
    if len(sys.argv) > 2:
        Path(sys.argv[2]).write_text(text)
    print(text)
    return 0


if __name__ == "__main__":
    sys.exit(main())
