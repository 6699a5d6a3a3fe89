# quick check of a kernel change: the parity tests of the push and one
# bench line.  usage (gpurun): bash tools/gpu_quick.sh <tag> [bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-quick}; shift
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > $O/bench.json 2> $O/bench.err &&
python3 -c "
import json; r=json.load(open('$O/bench.json')); k=r['kernels']
print('value %.4g  ms/step %.2f  solve %.2f  push %.3f ms frac %.3f' % (r['value'], r['ms_per_step'], r['poisson_ms_per_step'], k['push']['mean_launch_ms'], k['push']['frac']))"
