#!/usr/bin/env python3
"""Summarise rocprofv3 output of a bench run into profiles/.

    python tools/pmc_summary.py <tag> <prof_dir> <pmc_fetch_dir> <pmc_write_dir>

Reads the rocpd databases (bench_results.db, rocprofv3's default output in
ROCm 7.2) or the CSV files (--output-format csv) that tools/profile_bench.sh
leaves under gpurun_out/, and writes

  profiles/<tag>_kernel_stats.csv   the --kernel-trace --stats summary
                                    (per kernel: calls, total/avg/min/max ns)
  profiles/<tag>_hbm_traffic.json   HBM bytes per launch of each kernel,
                                    corrected as MI355X_MICROARCH.md prescribes
                                    for gfx950: counters are in KiB; FETCH_SIZE
                                    reports half of the bytes of wide coalesced
                                    reads, so it is doubled; WRITE_SIZE is taken
                                    as is; the two come from separate passes.
"""
import csv
import json
import re
import sqlite3
import sys
from collections import defaultdict
from pathlib import Path


def short(name: str) -> str:
    """'void (anonymous namespace)::k_accel<3, true, true>(double const*, ...)' -> 'k_accel<3, true, true>'"""
    s = re.sub(r"^void ", "", name)
    s = re.sub(r"\(anonymous namespace\)::", "", s)
    depth, out = 0, []
    for ch in s:
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out).strip()


def stats(d: Path) -> list:
    db = d / "bench_results.db"
    rows = []
    if db.exists():
        c = sqlite3.connect(db)
        per = defaultdict(list)
        for name, dur in c.execute("select name, duration from kernels"):
            per[short(name)].append(float(dur))
        tot = sum(sum(v) for v in per.values())
        for k, v in per.items():
            m = sum(v) / len(v)
            sd = (sum((x - m) ** 2 for x in v) / len(v)) ** 0.5
            rows.append([k, len(v), sum(v), m, 100.0 * sum(v) / tot, min(v), max(v), sd])
    else:
        for r in csv.DictReader(open(d / "bench_kernel_stats.csv")):
            rows.append([short(r["Name"]), int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"]),
                         float(r["Percentage"]), float(r["MinNs"]), float(r["MaxNs"]), float(r["StdDev"])])
    rows.sort(key=lambda r: -r[2])
    return rows


def counters(d: Path, name: str) -> dict:
    per = defaultdict(list)
    db = d / "bench_results.db"
    if db.exists():
        c = sqlite3.connect(db)
        q = "select kernel_name, grid_size, value from counters_collection where counter_name=? order by dispatch_id"
        for k, g, v in c.execute(q, (name,)):
            per[(short(k), int(g))].append(float(v) * 1024.0)
    else:
        for r in csv.DictReader(open(d / "bench_counter_collection.csv")):
            if r["Counter_Name"] == name:
                per[(short(r["Kernel_Name"]), int(r["Grid_Size"]))].append(float(r["Counter_Value"]) * 1024.0)
    return per


def main() -> int:
    tag, prof, fetch, write = sys.argv[1], Path(sys.argv[2]), Path(sys.argv[3]), Path(sys.argv[4])
    out = Path(__file__).resolve().parent.parent / "profiles"
    out.mkdir(exist_ok=True)
    with open(out / f"{tag}_kernel_stats.csv", "w", newline="") as fh:
        w = csv.writer(fh, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        for r in stats(prof):
            w.writerow(r)
    f, wr = counters(fetch, "FETCH_SIZE"), counters(write, "WRITE_SIZE")
    res = {"_note": "HBM bytes per launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes); "
                    "FETCH_SIZE doubled and KiB->B per MI355X_MICROARCH.md -- see tools/pmc_summary.py",
           "kernels": []}
    for k in sorted(set(f) | set(wr)):
        fb = [2.0 * x for x in f.get(k, [])]
        wb = wr.get(k, [])
        m = {"name": k[0], "grid_size": k[1], "launches": max(len(fb), len(wb)),
             "fetch_bytes_per_launch_mean": sum(fb) / len(fb) if fb else None,
             "write_bytes_per_launch_mean": sum(wb) / len(wb) if wb else None,
             "fetch_bytes_per_launch": fb[:64], "write_bytes_per_launch": wb[:64]}
        if fb and wb:
            m["traffic_bytes_per_launch_mean"] = m["fetch_bytes_per_launch_mean"] + m["write_bytes_per_launch_mean"]
        res["kernels"].append(m)
    (out / f"{tag}_hbm_traffic.json").write_text(json.dumps(res, indent=1))
    for m in res["kernels"]:
        if m["grid_size"] > 1 << 20:
            print(m["name"], m["grid_size"], m["launches"], m.get("traffic_bytes_per_launch_mean"))
    return 0


if __name__ == "__main__":
    sys.exit(main())
