# round 6: E = -grad phi with one component per thread (contiguous stores;
# PINC_EFIELD_ELEMS, lib_ee) -- the step tests on it, then a C4 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r06aa
mkdir -p $O
PINC_LIBDIR=pinc_amd/lib_ee timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mg_sine.py -x -v --timeout 300 --timeout-method thread -m gpu > $O/tests_ee.log 2>&1 || { tail -40 $O/tests_ee.log; exit 1; }
tail -1 $O/tests_ee.log
bash tools/gpu_ab.sh r06aa_efield_elems base:pinc_amd/lib ee:pinc_amd/lib_ee base2:pinc_amd/lib ee2:pinc_amd/lib_ee -- --steps 20 --warmup 3
