# sort-trigger probe: per-push displaced fraction and mean block cell box
# (PINC_TRACE_SORT=1) for C4 and C4 two-stream, then bench lines of both
# with population:sortSpread values.  usage (gpurun): bash tools/sort_spread_probe.sh <tag> [spread...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export PINC_QUIET=1
T=${1:-spread}; shift
O=gpurun_out/$T
mkdir -p $O
for w in c4 c4ts; do
  PINC_TRACE_SORT=1 timeout -k 10 300 python -u bench.py --workload $w --steps 24 --warmup 1 --no-cpu-baseline > $O/trace_$w.json 2> $O/trace_$w.err || { tail -5 $O/trace_$w.err; exit 1; }
  grep "cell box" $O/trace_$w.err > $O/trace_$w.txt
done
for sp in 0 "$@"; do
  for w in c4ts c4; do
    timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --sort-spread $sp > $O/bench_${w}_$sp.json 2> $O/bench_${w}_$sp.err || { tail -5 $O/bench_${w}_$sp.err; exit 1; }
    python3 -c "
import json; r=json.load(open('$O/bench_${w}_$sp.json')); k=r['push_kinds']
print('$w spread $sp: %.4g G/s %.2f ms/step solve %.2f sort %d count %d plain %d (%.2f/%.2f/%.2f ms)' % (r['value']/1e9, r['ms_per_step'], r['poisson_ms_per_step'], k['push_sort']['launches'], k['push_count']['launches'], k['push_plain']['launches'], k['push_sort']['mean_launch_ms'], k['push_count']['mean_launch_ms'], k['push_plain']['mean_launch_ms']))" | tee -a $O/summary.txt
  done
done
