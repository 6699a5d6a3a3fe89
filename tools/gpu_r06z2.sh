# round 6: C2 without the profiler, 200 steps: the bench default (one
# workgroup per solve) against the per-level graph path, twice each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r06z2
mkdir -p $O
for r in 1 2; do
  for v in 1 0; do
    PINC_MG_SMALL=$v timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --workload c2 --steps 200 --warmup 20 > $O/c2_small${v}_$r.json 2> $O/c2_small${v}_$r.err || { tail -20 $O/c2_small${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c2_small${v}_$r.json')); print('small=$v run $r', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],4), 'ms/step solve', round(d['poisson_ms_per_step'],4), 'cycles', d['mg_cycles_per_solve'])"
  done
done
