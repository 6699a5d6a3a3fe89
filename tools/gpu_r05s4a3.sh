# k_gs_sweep4c with the rho ring: planes fetched 3 steps ahead (lib_s4a3)
# against 2: the sweep tests on the variant, then a bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05s4a3
mkdir -p $O
PINC_LIBDIR=pinc_amd/lib_s4a3 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab.sh r05s4a3_ab a2:pinc_amd/lib a3:pinc_amd/lib_s4a3 a2b:pinc_amd/lib a3b:pinc_amd/lib_s4a3 -- --steps 10 --warmup 3
