# round 6: the counting push with one LDS atomic per thread run
# (PINC_PUSH_COUNT_RUNS, lib_cr) and nontemporal stores in the sorting push
# (PINC_PUSH_SORT_NT, lib_snt): the bench-flag parity tests on each variant,
# then an A/B against the default library
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r06i
mkdir -p $O
for L in lib_cr lib_snt; do
  PINC_LIBDIR=pinc_amd/$L timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -x -v --timeout 300 --timeout-method thread -m gpu > $O/tests_$L.log 2>&1 || { tail -40 $O/tests_$L.log; exit 1; }
  tail -1 $O/tests_$L.log
done
bash tools/gpu_ab.sh r06i_count_sort base:pinc_amd/lib cr:pinc_amd/lib_cr snt:pinc_amd/lib_snt base2:pinc_amd/lib -- --steps 50 --warmup 5
