# one bench per value of a bench.py option.
# usage (gpurun): bash tools/gpu_argsweep.sh <tag> <--option> <v1> <v2> ... [-- other bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; OPT=$2; shift 2
O=gpurun_out/$T
mkdir -p $O
vals=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do vals+=("$1"); shift; done
[ "$1" == "--" ] && shift
for x in "${vals[@]}"; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline $OPT $x "$@" > $O/$x.json 2> $O/$x.err || exit 1
  python3 -c "
import json; r=json.load(open('$O/$x.json')); k=r['kernels']
print('%s %-8s value %.4g ms/step %.2f solve %.2f push-phase %.2f push %.3f ms' % ('$OPT', '$x', r['value'], r['ms_per_step'], r['poisson_ms_per_step'], r['push_deposit_ms_per_step'], k['push']['mean_launch_ms']))" | tee -a $O/summary.txt
done
