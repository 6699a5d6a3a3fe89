# round 6: contiguous push loads/stores with the adjacent-lane exchange
# (PINC_PUSH_XCH) -- push parity tests, then an A/B against the round-5
# mapping (pinc_amd/lib_x, built with -DPINC_PUSH_XCH=0)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r06d
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_reference_kat.py tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_langmuir.py -x -v --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
AB_PMC=1 bash tools/gpu_ab.sh r06d_xch r05map:pinc_amd/lib_x xch:pinc_amd/lib -- --steps 30 --warmup 3
