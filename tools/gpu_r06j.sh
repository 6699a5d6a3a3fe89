# round 6: the sorting push's item pairs (PINC_PUSH_SORT_PAIRS, lib_sp) --
# the sorting-push parity tests on the variant, then an A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r06j
mkdir -p $O
PINC_LIBDIR=pinc_amd/lib_sp timeout -k 10 800 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu > $O/tests_sp.log 2>&1 || { tail -40 $O/tests_sp.log; exit 1; }
tail -1 $O/tests_sp.log
bash tools/gpu_ab.sh r06j_sortpairs base:pinc_amd/lib sp:pinc_amd/lib_sp base2:pinc_amd/lib sp2:pinc_amd/lib_sp -- --steps 50 --warmup 5
