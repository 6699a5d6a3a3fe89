set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05f
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reference_kat.py tests/test_gpu_errors.py tests/test_gpu_mg_scale.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/r05f/tests.log 2>&1 || { tail -30 gpurun_out/r05f/tests.log; exit 1; }
tail -2 gpurun_out/r05f/tests.log
bash tools/gpu_ab.sh r05f base:pinc_amd/lib_base nospec:pinc_amd/lib:PINC_MG_SPECULATE=0 new:pinc_amd/lib -- --steps 10 --warmup 3
