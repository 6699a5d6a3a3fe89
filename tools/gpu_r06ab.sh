# round 6: E's negation (gMul(E, -1)) inside the finite-difference pass of
# regular()'s step -- its bit-identity test and the step parity tests, then
# a C4 A/B against the previous library
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r06ab
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_langmuir.py tests/test_gpu_mg_shard.py tests/test_gpu_objects.py -x -v --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab.sh r06ab_efield_neg old:pinc_amd/lib_old new:pinc_amd/lib old2:pinc_amd/lib_old new2:pinc_amd/lib -- --steps 20 --warmup 3
