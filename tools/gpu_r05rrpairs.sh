# level-0 residual + restriction on x pairs (default) against single loads
# (lib_rrold): kernel and MG tests, then a bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05rrpairs
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_mg_scale.py tests/test_gpu_mg_sine.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab.sh r05rrpairs_ab pairs:pinc_amd/lib old:pinc_amd/lib_rrold pairs2:pinc_amd/lib old2:pinc_amd/lib_rrold -- --steps 10 --warmup 3
