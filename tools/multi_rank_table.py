#!/usr/bin/env python3
"""Print the multi-rank diagnostic block of bench.py lines (N > 1): phases
(max over ranks), collectives by kind (bytes, calls and ms per step, max over
ranks) and each rank's dominant-kernel roofline.

    python tools/multi_rank_table.py gpurun_out/<tag>/c4_n4.json [...]
"""
import json
import sys


def main() -> int:
    for path in sys.argv[1:]:
        r = json.loads(open(path).read())
        m = r.get("multi_rank")
        print(f"== {path}: {r['config'].get('workload')} n_gpus {r['n_gpus']} value {r['value']:.4g} "
              f"ms/step {r['ms_per_step']:.2f} solve {r.get('poisson_ms_per_step', 0):.2f} "
              f"cycles/solve {r.get('mg_cycles_per_solve')}")
        if not m:
            print("   (no multi_rank block)")
            continue
        print(f"   transport {m['transport']}, ranks {m['ranks']}")
        ph = m["phase_ms_per_step_max"]
        print("   phases (ms/step, max over ranks): " + ", ".join(f"{k} {v:.2f}" for k, v in ph.items()))
        print(f"   {'collective':<20}{'MB/step/rank':>14}{'calls/step':>12}{'ms/step max':>13}")
        for k, c in m["comm_per_step"].items():
            print(f"   {k:<20}{c['bytes_per_step_per_rank_max'] / 1e6:>14.3f}{c['calls_per_step']:>12.2f}"
                  f"{c['ms_per_step_max']:>13.3f}")
        for p in m.get("per_rank", []):
            rf = p.get("roofline")
            if rf:
                print(f"   rank {p['rank']}: {p['particles']} particles, {rf['kernel']} {rf['mean_launch_ms']:.3f} ms "
                      f"= {rf['achieved_GBs']:.0f} GB/s ({rf['frac']:.3f})")
    return 0


if __name__ == "__main__":
    sys.exit(main())
