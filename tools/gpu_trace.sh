# phase trace of the push (PINC_TRACE_SORT=2) over a steady-state run.
# usage (gpurun): bash tools/gpu_trace.sh <tag> [bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
export PINC_QUIET=1
T=${1:-trace}; shift
O=gpurun_out/$T
mkdir -p $O
PINC_TRACE_SORT=2 timeout -k 10 300 python -u bench.py --steps ${TRACE_STEPS:-30} --warmup 2 --no-cpu-baseline "$@" > $O/trace.json 2> $O/trace.err || { tail -5 $O/trace.err; exit 1; }
grep "push species" $O/trace.err > $O/push_trace.txt; tail -24 $O/push_trace.txt
