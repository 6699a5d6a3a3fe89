set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r05x
mkdir -p $O
PINC_LIBDIR=pinc_amd/lib_ci timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_ab.sh r05x base:pinc_amd/lib ci:pinc_amd/lib_ci -- --steps 20 --warmup 3 || exit 1
