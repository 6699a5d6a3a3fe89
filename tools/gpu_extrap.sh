set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02ah
for e in 0 1; do
PINC_VERBOSE=1 timeout -k 10 300 python -u bench.py --steps 40 --warmup 12 --no-cpu-baseline --mg-extrapolate $e > gpurun_out/r02ah/b$e.json 2> gpurun_out/r02ah/b$e.err || exit 1
python3 -c "
import json; r=json.load(open('gpurun_out/r02ah/b$e.json'))
print('extrap $e value %.4g ms/step %.2f solve %.2f cycles %.2f' % (r['value'], r['ms_per_step'], r['poisson_ms_per_step'], r['mg_cycles_per_solve']))"
done
grep "solve cycle" gpurun_out/r02ah/b1.err | tail -8
