set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r05ac
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_reference_kat.py tests/test_gpu_multirank.py tests/test_gpu_objects.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_ab.sh r05ac nobox:pinc_amd/lib_nobox box:pinc_amd/lib -- --steps 20 --warmup 3 || exit 1
