# one short bench per value of an environment variable.
# usage (gpurun): bash tools/gpu_envsweep.sh <tag> <VAR> <v1> <v2> ... [-- bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; V=$2; shift 2
O=gpurun_out/$T
mkdir -p $O
vals=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do vals+=("$1"); shift; done
[ "$1" == "--" ] && shift
for x in "${vals[@]}"; do
  env $V=$x timeout -k 10 240 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline "$@" > $O/$x.json 2> $O/$x.err || exit 1
  python3 -c "
import json; r=json.load(open('$O/$x.json')); k=r['kernels']
print('%s=%-10s value %.4g ms/step %.2f solve %.2f cycles %.1f push %.3f ms' % ('$V', '$x', r['value'], r['ms_per_step'], r['poisson_ms_per_step'], r['mg_cycles_per_solve'], k['push']['mean_launch_ms']))" | tee -a $O/summary.txt
done
