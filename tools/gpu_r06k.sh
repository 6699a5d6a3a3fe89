# round 6: the one-workgroup small solve (multigrid:oneCU / PINC_MG_SMALL) --
# its parity test, the 2-D oracle tests and C2's Langmuir tests forced onto
# it, then C2 A/B against the spectral-coarse graph path
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r06k
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_mg_scale.py -x -v --timeout 200 --timeout-method thread -m gpu -k "one_cu or nd_solve" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
PINC_MG_SMALL=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_langmuir.py tests/test_gpu_mg_scale.py tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu -k "c2" > $O/tests_forced.log 2>&1 || { tail -40 $O/tests_forced.log; exit 1; }
tail -1 $O/tests_forced.log
bash tools/gpu_ab.sh r06k_c2small base:pinc_amd/lib small:pinc_amd/lib:PINC_MG_SMALL=1 -- --workload c2 --steps 200 --warmup 20
for sm in 2,2 3,3 4,4 6,6; do
  PINC_MG_SMALL=1 timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --workload c2 --steps 200 --warmup 20 --mg-smooth $sm > $O/small_$sm.json 2> $O/small_$sm.err || { tail -20 $O/small_$sm.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/small_$sm.json')); print('$sm', d['ms_per_step'], d['poisson_ms_per_step'], d['mg_cycles_per_solve'])"
done
