# the smoother's XCD-contiguous tile order (PINC_MG_XCD=1, lib_t16)
# re-measured with the rho ring (two workgroups per CU): sweep tests on the
# variant, then a bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05t16
mkdir -p $O
PINC_LIBDIR=pinc_amd/lib_t16 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab.sh r05t16_ab base:pinc_amd/lib t16:pinc_amd/lib_t16 base2:pinc_amd/lib t162:pinc_amd/lib_t16 -- --steps 10 --warmup 3
