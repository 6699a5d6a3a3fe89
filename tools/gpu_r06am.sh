# round 6: the cell-ranked sorting push's cell offsets by a 16-lane scan
# per brick (was one thread per brick, 16 dependent LDS steps) -- C4 A/B
# against the previous library, then the push parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
bash tools/gpu_ab.sh r06am_cellrank_scan old:pinc_amd/lib_old new:pinc_amd/lib old2:pinc_amd/lib_old new2:pinc_amd/lib || exit 1
O=gpurun_out/r06am_cellrank_scan
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_langmuir.py tests/test_gpu_objects.py tests/test_gpu_scale.py tests/test_gpu_multirank.py -x -v --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
