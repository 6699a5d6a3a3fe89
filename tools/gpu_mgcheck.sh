# multigrid change check: the MG parity tests, then the C2 line and the
# rep256 probe.  usage (gpurun): bash tools/gpu_mgcheck.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export PINC_QUIET=1
O=gpurun_out/${1:-mgcheck}
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests/test_gpu_mg_scale.py tests/test_gpu_mg_shard.py tests/test_gpu_langmuir.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench.py --workload c2 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || exit 1
python3 -c "
import json; r=json.load(open('$O/bench_c2.json'))
print('c2 value %.4g ms/step %.2f solve %.2f' % (r['value'], r['ms_per_step'], r['poisson_ms_per_step']))"
timeout -k 10 200 python -u tools/mg_shard_probe.py --cases rep256 --out $O/probe.json > $O/probe.log 2>&1 || exit 1
grep -o '"ms_per_cycle": [0-9.]*' $O/probe.log
