# multigrid level-kernel experiment: MG GPU tests, then C4 and C2 bench lines
# with and without the V-cycle graph, and the C4 kernel statistics.
# usage (gpurun): bash tools/gpu_mgab.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/${1:-mgab}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_mg_scale.py tests/test_gpu_mg_shard.py tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for a in "--workload c2" "--workload c2 --mg-graph 1" "" "--mg-graph 1"; do
  n=$(echo "x$a" | tr -d ' -')
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline $a > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
  python3 -c "
import json; r=json.load(open('$O/$n.json'))
print('%-32s value %.4g ms/step %.2f solve %.2f cycles %.2f' % ('$a', r['value'], r['ms_per_step'], r['poisson_ms_per_step'], r['mg_cycles_per_solve']))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof.json 2> $O/prof.err || exit 1
python3 tools/db_stats.py $O/prof $O/kernel_stats.csv && rm -rf $O/prof
