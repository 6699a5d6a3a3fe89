# round 6: the push's lane exchange, row form (PINC_PUSH_XCH 2: rows of 16
# lanes keep 64 consecutive particles) -- parity tests, then an A/B of the
# round-5 mapping (lib_x), the adjacent-lane exchange (lib_1), the row
# exchange (lib) and the row exchange with word-wise E staging (lib_e)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r06e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_reference_kat.py tests/test_gpu_parity.py tests/test_gpu_flag_switches.py -x -v --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
AB_PMC=1 bash tools/gpu_ab.sh r06e_xch r05map:pinc_amd/lib_x xch1:pinc_amd/lib_1 xch2:pinc_amd/lib xch2e:pinc_amd/lib_e -- --steps 30 --warmup 3
