# round 6: the sort trigger's fraction at C4 after the round-6 push (bench
# lines without the profiler, 50 steps after 5)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r06p
mkdir -p $O
for f in 0.8 0.5 0.65 1.0 0.8; do
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --sort-fraction $f > $O/c4_sf$f.json 2> $O/c4_sf$f.err || { tail -20 $O/c4_sf$f.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/c4_sf$f.json')); k=d['push_kinds']
print('sort-fraction $f', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],3), 'ms/step; plain', round(k['push_plain']['mean_launch_ms'],2), 'x', k['push_plain']['launches'], 'count', round(k.get('push_count',{}).get('mean_launch_ms',0),2), 'x', k.get('push_count',{}).get('launches',0), 'sort', round(k.get('push_sort',{}).get('mean_launch_ms',0),2), 'x', k.get('push_sort',{}).get('launches',0), [(s['species'], round(s['plain_ms'],2), s['sorts']) for s in k['by_species']])"
done
