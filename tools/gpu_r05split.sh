# the smoother's XCD-contiguous tile order (PINC_MG_XCD=1, lib_nosplit)
# re-measured with the rho ring (two workgroups per CU): sweep tests on the
# variant, then a bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05split
mkdir -p $O
PINC_LIBDIR=pinc_amd/lib_nosplit timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab.sh r05split_ab base:pinc_amd/lib merged:pinc_amd/lib_nosplit base2:pinc_amd/lib merged2:pinc_amd/lib_nosplit -- --steps 10 --warmup 3
