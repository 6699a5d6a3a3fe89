#!/usr/bin/env python3
"""Side-by-side summary of tools/gpu_ab.sh runs.

    python tools/ab_table.py <out_dir> <libdir>...

For each variant: the bench line's value, ms/step, solve and push-kind
times, then the average duration of the kernels that take the most time
(rocprofv3 --kernel-trace --stats, tools/db_stats.py) in each variant, and
the PMC traffic per launch of the push and the smoother when present.
"""
import csv
import json
import sys
from pathlib import Path


def main() -> int:
    out = Path(sys.argv[1])
    names = [Path(p).name for p in sys.argv[2:]]
    stats, lines = {}, {}
    for n in names:
        try:
            lines[n] = json.loads((out / f"{n}.json").read_text().strip().splitlines()[-1])
        except (OSError, ValueError, IndexError):
            lines[n] = None
        rows = {}
        f = out / f"{n}_kernel_stats.csv"
        if f.exists():
            for r in csv.DictReader(open(f)):
                name = r["Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
                rows[name] = (int(r["Calls"]), float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6)
        stats[n] = rows
    for n in names:
        r = lines[n]
        if not r:
            print(f"{n}: no bench line")
            continue
        pk = r.get("push_kinds", {})
        kinds = " ".join(f"{k}={v['mean_launch_ms']:.2f}ms x{v['launches']}" for k, v in pk.items()
                         if isinstance(v, dict))
        for row in pk.get("by_species", []):
            kinds += (f" | s{row['species']}: plain {row['plain_ms'] or 0:.2f} fresh {row['fresh_plain_ms'] or 0:.2f}"
                      f" count {row['count_ms'] or 0:.2f} sort {row['sort_ms'] or 0:.2f}")
        print(f"{n}: value {r['value']:.4g} ms/step {r['ms_per_step']:.2f} solve {r['poisson_ms_per_step']:.2f} "
              f"push frac {r['roofline']['frac']:.3f} {kinds}")
    top = set()
    for n in names:
        top |= {k for k, _ in sorted(stats[n].items(), key=lambda kv: -kv[1][2])[:14]}
    print("%-60s" % "kernel (avg ms, calls)" + "".join("%22s" % n for n in names))
    for k in sorted(top, key=lambda k: -max(stats[n].get(k, (0, 0, 0))[2] for n in names)):
        cells = []
        for n in names:
            c = stats[n].get(k)
            cells.append("%22s" % (f"{c[1]:.4f} x{c[0]}" if c else "-"))
        print("%-60s" % k[:60] + "".join(cells))
    for n in names:
        f = out / f"{out.name}_{n}_hbm_traffic.json"
        if f.exists():
            d = json.loads(f.read_text())
            for k in d["kernels"]:
                if k.get("traffic_bytes_per_launch_mean") and k["grid_size"] >= 1 << 20 and (
                        k["name"].startswith("k_push") or k["name"].startswith("k_gs_sweep")):
                    print(f"  {n} {k['name']}: fetch {k['fetch_bytes_per_launch_mean'] / 1e9:.3f} GB "
                          f"write {k['write_bytes_per_launch_mean'] / 1e9:.3f} GB per launch")
    return 0


if __name__ == "__main__":
    sys.exit(main())
