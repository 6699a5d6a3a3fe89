# per-dispatch push durations in order (the decay between sorts) for one or
# more library variants: rocprofv3 --kernel-trace of a bench run, then
# tools/trace_summary.py (kernel totals + the k_push sequence).
# usage (gpurun): bash tools/gpu_push_seq.sh <tag> <name:libdir>... [-- bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
T=$1; shift
O=gpurun_out/$T
mkdir -p $O
libs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do libs+=("$1"); shift; done
[ "$1" == "--" ] && shift
for V in "${libs[@]}"; do
  IFS=: read -r n L <<< "$V"
  PINC_LIBDIR=$L timeout -k 10 500 rocprofv3 --kernel-trace -d $O/prof_$n -o run -- \
    python3 -u bench.py --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 tools/trace_summary.py $O/prof_$n 24 > $O/${n}_seq.txt && rm -rf $O/prof_$n
  python3 -c "
import json; r=json.load(open('$O/$n.json'))
print('$n value %.4g ms/step %.2f solve %.2f push %.2f' % (r['value'], r['ms_per_step'], r['poisson_ms_per_step'], r['push_deposit_ms_per_step']), {k: round(v['mean_launch_ms'], 2) for k, v in r['push_kinds'].items() if isinstance(v, dict)})"
done
