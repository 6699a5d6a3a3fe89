set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05b
PINC_LIBDIR=pinc_amd/lib_unfixed timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k literal_loop_tiled -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/r05b/unfixed.log 2>&1
echo "unfixed rc=$?"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_c_driver.py tests/test_gpu_reference_kat.py -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/r05b/fixed.log 2>&1
rc=$?
tail -5 gpurun_out/r05b/fixed.log
exit $rc
