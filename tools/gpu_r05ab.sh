set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ab
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_mg_scale.py tests/test_gpu_mg_shard.py tests/test_gpu_errors.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
