# object tests, then the C5 bench line (fused collection).  usage (gpurun): bash tools/gpu_c5.sh <tag> [bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-c5}; shift
O=gpurun_out/$T
mkdir -p $O
export PINC_QUIET=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_objects.py -x -v --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python -u bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline "$@" > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
python3 -c "
import json; r=json.load(open('$O/bench_c5.json'))
print('C5 value %.4g ms/step %.2f solve %.2f phases %s' % (r['value'], r['ms_per_step'], r['poisson_ms_per_step'], {k: round(v,2) for k,v in r['phase_ms_per_step'].items()}))"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 1; }
python3 -c "
import json; r=json.load(open('$O/bench_c4.json'))
print('C4 value %.4g ms/step %.2f solve %.2f phases %s' % (r['value'], r['ms_per_step'], r['poisson_ms_per_step'], {k: round(v,2) for k,v in r['phase_ms_per_step'].items()}))"
