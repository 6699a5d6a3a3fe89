# time the push of several in-tree library variants (PINC_LIBDIR) with one
# short bench each.  usage (gpurun): bash tools/gpu_variants.sh <tag> <libdir>... [-- bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; shift
O=gpurun_out/$T
mkdir -p $O
libs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do libs+=("$1"); shift; done
[ "$1" == "--" ] && shift
for L in "${libs[@]}"; do
  n=$(basename $L)
  PINC_LIBDIR=$L timeout -k 10 240 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || exit 1
  python3 -c "
import json; r=json.load(open('$O/$n.json')); k=r['kernels']
print('%-14s value %.4g ms/step %.2f solve %.2f push %.3f ms frac %.3f' % ('$n', r['value'], r['ms_per_step'], r['poisson_ms_per_step'], k['push']['mean_launch_ms'], k['push']['frac']))" | tee -a $O/summary.txt
done
