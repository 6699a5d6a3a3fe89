# steady-state sort schedule sweep: 40 timed steps after 12 warm-up steps.
# usage (gpurun): bash tools/gpu_sortsweep.sh <tag> "<bench args>"...
set -o pipefail
cd $GRAFT_REPO_ROOT
export PINC_QUIET=1
T=$1; shift
O=gpurun_out/$T
mkdir -p $O
i=0
for args in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --steps 40 --warmup 12 --no-cpu-baseline $args > $O/b$i.json 2> $O/b$i.err || { tail -5 $O/b$i.err; exit 1; }
  python3 -c "
import json; r=json.load(open('$O/b$i.json')); k=r['kernels']
print('%-40s value %.4g ms/step %.2f solve %.2f push %.2f' % ('$args', r['value'], r['ms_per_step'], r['poisson_ms_per_step'], k['push']['mean_launch_ms']))" | tee -a $O/summary.txt
done
