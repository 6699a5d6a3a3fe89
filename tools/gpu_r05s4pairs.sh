# k_gs_sweep4c with 16-B x-pair fetches of phi and rho (default) against
# three 8-B loads (lib_s4nopair): sweep/MG tests, then a bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05s4pairs
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_mg_scale.py tests/test_gpu_mg_sine.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab.sh r05s4pairs_ab pairs:pinc_amd/lib nopair:pinc_amd/lib_s4nopair pairs2:pinc_amd/lib nopair2:pinc_amd/lib_s4nopair -- --steps 10 --warmup 3
