# round 6: the small solve's kernel tests, its phase times (diagnostic
# build lib_sd), and C2 with it against the per-level path
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r06l
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -m gpu -k "small" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for sp in 1; do
  PINC_LIBDIR=pinc_amd/lib_sd timeout -k 10 120 python3 -u tools/small_solve_diag.py --size 128 --spectral $sp > $O/diag_$sp.txt 2>&1 || { tail -20 $O/diag_$sp.txt; exit 1; }
  cat $O/diag_$sp.txt
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_mg_scale.py -x -v --timeout 200 --timeout-method thread -m gpu -k "one_cu or nd_solve" > $O/tests_mg.log 2>&1 || { tail -40 $O/tests_mg.log; exit 1; }
tail -1 $O/tests_mg.log
for sm in 2,2 4,4; do
  for v in 0 1; do
    PINC_MG_SMALL=$v timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --workload c2 --steps 200 --warmup 20 --mg-smooth $sm > $O/c2_${v}_$sm.json 2> $O/c2_${v}_$sm.err || { tail -20 $O/c2_${v}_$sm.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c2_${v}_$sm.json')); print('small=$v $sm', d['ms_per_step'], d['poisson_ms_per_step'], d['mg_cycles_per_solve'])"
  done
done
