set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05i
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reference_kat.py tests/test_gpu_scale.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r05i/tests.log 2>&1 || { tail -30 gpurun_out/r05i/tests.log; exit 1; }
tail -2 gpurun_out/r05i/tests.log
bash tools/pmc_push.sh r05i_pmc
