# round 6, first call: the extraction known answer through the HIP path, then
# a short C4 bench (probe launch counts of the smoother)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_reference_kat.py -x -v --timeout 120 --timeout-method thread -m gpu > $O/kat.log 2>&1 || { tail -40 $O/kat.log; exit 1; }
tail -3 $O/kat.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; r=json.load(open('$O/bench.json'))
print('value %.4g ms/step %.2f solve %.2f cycles/solve %.2f' % (r['value'], r['ms_per_step'], r['poisson_ms_per_step'], r['mg_cycles_per_solve']))
for k,v in r['kernels'].items(): print(k, v['launches'], v['samples'], '%.4f'%v['mean_launch_ms'], '%.3f'%v['est_ms_per_step'])
"
