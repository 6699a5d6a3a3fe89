# round 6: the C4 bench line over 300 timed steps (steady state, energy
# history) and the default 50-step line again, on the final tree
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r06long
mkdir -p $O
timeout -k 10 600 python -u bench.py --steps 300 --warmup 5 --no-cpu-baseline > $O/bench_c4_300.json 2> $O/bench_c4_300.err || { tail -20 $O/bench_c4_300.err; exit 1; }
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $O/bench_c4_50.json 2> $O/bench_c4_50.err || { tail -20 $O/bench_c4_50.err; exit 1; }
for f in bench_c4_300 bench_c4_50; do python3 -c "
import json; r=json.load(open('$O/$f.json'))
print('$f', 'value %.4g ms/step %.2f solve %.2f push %.2f frac %.3f' % (r['value'], r['ms_per_step'], r['poisson_ms_per_step'], r['roofline']['mean_launch_ms'], r['roofline']['frac']), json.dumps(r.get('energy'))[:300])"; done
