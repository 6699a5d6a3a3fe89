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

    python tools/pmc_summary.py <tag> <prof_dir> <pmc_fetch_dir> <pmc_write_dir> [<bench.json>]

The optional bench line (the profiled command's output) gives the traffic
file its "config" (bench.py's traffic_key: workload, grid, ppc, GPU count,
layout); bench.py reports traffic only from a profile of its own config.

    python tools/pmc_summary.py --calibrate <tag> <calibration_dir>

reads tools/pmc_calibrate.sh's output (rates.jsonl + FETCH_SIZE / WRITE_SIZE
passes of tools/pmc_calibrate.hip, whose kernels touch known byte counts in
the access patterns of this repository's kernels) and writes
profiles/<tag>_pmc_calibration.json: counter bytes / true bytes per pattern.
The FETCH_SIZE correction of a kernel is then 1 / (that ratio) for the
pattern its HBM reads have (FETCH_PATTERN below); without a calibration
file the guide's x2 is used for every kernel.
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


def _db(d: Path) -> Path:
    """rocprofv3's rocpd database of a run (<output name>_results.db)."""
    dbs = sorted(d.glob("*_results.db"))
    return dbs[0] if dbs else d / "bench_results.db"


def stats(d: Path) -> list:
    db = _db(d)
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
    db = _db(d)
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


# the calibration pattern of each kernel's HBM reads (tools/pmc_calibrate.hip)
FETCH_PATTERN = [
    ("k_push", "rd_pair32"), ("k_accel", "rd_pair32"), ("k_move_classify", "rd_pair32"), ("k_deposit", "rd_pair32"),
    ("k_gs_", "rd_b64_rows"), ("k_residual", "rd_b64_rows"), ("k_restrict", "rd_b64_rows"),
    ("k_prolong", "rd_b64_rows"), ("k_efield", "rd_b64_rows"), ("k_extrapolate", "rd_b64"),
]
PROFILES = Path(__file__).resolve().parent.parent / "profiles"


def calibration():
    """Newest profiles/*_pmc_calibration.json: {pattern: fetch counter/true}."""
    files = sorted(PROFILES.glob("*_pmc_calibration.json"))
    if not files:
        return None, None
    d = json.loads(files[-1].read_text())
    return {k: v["fetch_ratio"] for k, v in d["patterns"].items() if v.get("fetch_ratio")}, files[-1].name


def fetch_factor(name: str, cal) -> tuple:
    if cal:
        for prefix, pat in FETCH_PATTERN:
            if name.startswith(prefix) and pat in cal:
                return 1.0 / cal[pat], pat
        if "rd_b128" in cal and "rd_b128" in cal:
            return 1.0 / cal["rd_b128"], "rd_b128"
    return 2.0, "guide x2"


def calibrate(tag: str, d: Path) -> int:
    rates = {}
    for line in (d / "rates.jsonl").read_text().splitlines():
        r = json.loads(line)
        rates[r["kernel"]] = r
    f, w = counters(d / "fetch" if (d / "fetch").exists() else d, "FETCH_SIZE"), counters(d / "write", "WRITE_SIZE")
    pats = {}
    for k, r in rates.items():
        fb = [v for (n, g), vs in f.items() if n == k for v in vs]
        wb = [v for (n, g), vs in w.items() if n == k for v in vs]
        e = {"true_bytes": r["bytes"], "best_ms": r["best_ms"], "GBs": r["GBs"]}
        if fb:
            e["fetch_counter_bytes"] = sum(fb) / len(fb)
            if k.startswith("rd_") or k.startswith("cp_"):
                e["fetch_ratio"] = e["fetch_counter_bytes"] / (r["bytes"] / (2 if k.startswith("cp_") else 1))
        if wb:
            e["write_counter_bytes"] = sum(wb) / len(wb)
            if k.startswith("wr_") or k.startswith("at_") or k.startswith("cp_"):
                e["write_ratio"] = e["write_counter_bytes"] / (r["bytes"] / (2 if k.startswith("cp_") else 1))
        pats[k] = e
    out = {"_note": "rocprofv3 FETCH_SIZE / WRITE_SIZE (KiB -> B) of tools/pmc_calibrate.hip's kernels against the "
                    "bytes each touches once (2 GiB buffers, beyond the Infinity Cache); ratio = counter / true",
           "patterns": pats}
    (PROFILES / f"{tag}_pmc_calibration.json").write_text(json.dumps(out, indent=1))
    for k, e in pats.items():
        print(k, {x: round(y, 3) for x, y in e.items() if "ratio" in x or x == "GBs"})
    return 0


def main() -> int:
    if sys.argv[1] == "--calibrate":
        return calibrate(sys.argv[2], Path(sys.argv[3]))
    tag, prof, fetch, write = sys.argv[1], Path(sys.argv[2]), Path(sys.argv[3]), Path(sys.argv[4])
    bench = json.loads(Path(sys.argv[5]).read_text().strip().splitlines()[-1]) if len(sys.argv) > 5 else None
    out = PROFILES
    out.mkdir(exist_ok=True)
    cal, cal_src = calibration()
    with open(out / f"{tag}_kernel_stats.csv", "w", newline="") as fh:
        w = csv.writer(fh, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        for r in stats(prof):
            w.writerow(r)
    f, wr = counters(fetch, "FETCH_SIZE"), counters(write, "WRITE_SIZE")
    res = {"_note": "HBM bytes per launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes); KiB->B; "
                    "FETCH_SIZE scaled by the calibrated factor of the kernel's read pattern (fetch_correction; "
                    "MI355X_MICROARCH.md's x2 without a calibration) -- see tools/pmc_summary.py",
           "config": (bench.get("config") or {}).get("traffic_key") if bench else None,
           "calibration": cal_src,
           "kernels": []}
    for k in sorted(set(f) | set(wr)):
        fac, pat = fetch_factor(k[0], cal)
        fb = [fac * x for x in f.get(k, [])]
        wb = wr.get(k, [])
        m = {"name": k[0], "grid_size": k[1], "launches": max(len(fb), len(wb)),
             "fetch_correction": fac, "fetch_pattern": pat,
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
