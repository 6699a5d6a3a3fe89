"""One summary line per bench JSON file (the last line of each)."""
import json
import sys

for path in sys.argv[1:]:
    d = json.loads(open(path).read().strip().splitlines()[-1])
    pk = d.get("push_kinds", {})
    plain = pk.get("push_plain", {}).get("mean_launch_ms")
    print(f"{path}: {d['value'] / 1e9:.2f} G/s step {d['ms_per_step']:.3f} ms solve {d['poisson_ms_per_step']:.3f} ms"
          f" cycles {d.get('mg_cycles_per_solve', 0):.2f} push {d['roofline']['mean_launch_ms']:.3f} ms"
          + (f" plain {plain:.3f} ms" if plain else "")
          + f" efield+accel {d['phase_ms_per_step'].get('efield', 0) + d['phase_ms_per_step'].get('accelerate', 0):.3f} ms")
