#!/bin/bash
# C4 bench at several native-multigrid smoothing counts (--mg-smooth), one
# line each into $OUT/<pre>_<post>.json; stops at the first failing run.
OUT=${OUT:-gpurun_out/mg_smooth}
STEPS=${STEPS:-20}
mkdir -p "$OUT"
VARIANTS=${VARIANTS:-10,10 4,4 2,2 6,6 4,6}
for ps in $VARIANTS; do
	tag=${ps/,/_}
	echo "== $ps"
	timeout -k 10 240 python -u bench.py --steps "$STEPS" --warmup 5 --no-cpu-baseline --mg-smooth "$ps" $EXTRA \
		> "$OUT/$tag.json" 2> "$OUT/$tag.log" || exit $?
	python - "$OUT/$tag.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], "%.2f G/s" % (d["value"] / 1e9), "step %.3f ms" % d["ms_per_step"],
      "solve %.3f ms" % d["poisson_ms_per_step"], "cycles %.2f" % d["mg_cycles_per_solve"])
PY
done
