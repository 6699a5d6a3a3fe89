# plain (unprofiled) bench lines of the other workloads.  usage (gpurun): bash tools/gpu_lines.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export PINC_QUIET=1
O=gpurun_out/${1:-lines}
mkdir -p $O
for w in c3 c2 c5; do
  timeout -k 10 600 python -u bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
  python3 -c "
import json; r=json.load(open('$O/bench_$w.json'))
print('$w value %.4g ms/step %.2f solve %.2f' % (r['value'], r['ms_per_step'], r['poisson_ms_per_step']))"
done
