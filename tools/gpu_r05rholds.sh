# rho in an LDS ring in k_gs_sweep4c: the sweep and multigrid tests, then an
# A/B of the C4 bench against the gathering kernel (pinc_amd/lib_s4old)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05rholds
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_mg_scale.py tests/test_gpu_mg_sine.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab.sh r05rholds_ab new:pinc_amd/lib old:pinc_amd/lib_s4old new2:pinc_amd/lib old2:pinc_amd/lib_s4old -- --steps 10 --warmup 3
