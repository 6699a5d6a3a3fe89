# k_gs_sweep4w (512 threads per 32 x 8 tile, lib_s4wide) against
# k_gs_sweep4c (256): sweep/MG tests on the variant, then a bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05s4wide
mkdir -p $O
PINC_LIBDIR=pinc_amd/lib_s4wide timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_mg_scale.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab.sh r05s4wide_ab base:pinc_amd/lib wide:pinc_amd/lib_s4wide base2:pinc_amd/lib wide2:pinc_amd/lib_s4wide -- --steps 10 --warmup 3
