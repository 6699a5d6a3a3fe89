set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05j
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reference_kat.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/r05j/tests.log 2>&1 || { tail -30 gpurun_out/r05j/tests.log; exit 1; }
tail -2 gpurun_out/r05j/tests.log
bash tools/gpu_ab.sh r05j prev:pinc_amd/lib_prev new:pinc_amd/lib -- --steps 10 --warmup 3
