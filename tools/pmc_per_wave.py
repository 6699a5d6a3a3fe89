#!/usr/bin/env python3
"""Per-wave view of the push PMC passes (tools/pmc_push.sh): every counter of
every dispatch divided by its wave count, dispatches side by side.

    python tools/pmc_per_wave.py <dir with p0.csv p1.csv p2.csv> [dispatch ...]
"""
import csv
import sys
from pathlib import Path


def main() -> int:
    d = Path(sys.argv[1])
    data = {}
    for f in sorted(d.glob("p*.csv")):
        for r in csv.DictReader(open(f)):
            e = data.setdefault(r["dispatch"], {"kernel": r["kernel"]})
            e.update({k: float(v) for k, v in r.items() if k not in ("dispatch", "kernel")})
    sel = sys.argv[2:] or list(data)
    keys = sorted({k for v in data.values() for k in v if k != "kernel"})
    print("%-26s" % "counter / wave" + "".join("%12s" % s for s in sel))
    print("%-26s" % "kernel" + "".join("%12s" % data[s]["kernel"].split("<")[1][:10] for s in sel))
    for k in keys:
        print("%-26s" % k + "".join("%12.1f" % (data[s].get(k, 0) / max(1.0, data[s].get("SQ_WAVES", 1))) for s in sel))
    return 0


if __name__ == "__main__":
    sys.exit(main())
