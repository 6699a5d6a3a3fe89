# round 6: the sorting push orders each brick's run by cell
# (PINC_SORT_CELLRANK=1) -- C4 A/B over 100 steps (the sorts' effect on the
# order builds up over many sorts) against the previous library and the
# new one with the option off, then the push parity tests on the variant
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
bash tools/gpu_ab.sh r06ak_sort_cellrank old:pinc_amd/lib_old cr:pinc_amd/lib_cr off:pinc_amd/lib old2:pinc_amd/lib_old cr2:pinc_amd/lib_cr -- --steps 100 --warmup 5 || exit 1
O=gpurun_out/r06ak_sort_cellrank
PINC_LIBDIR=pinc_amd/lib_cr timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_langmuir.py tests/test_gpu_objects.py tests/test_gpu_scale.py -x -v --timeout 300 --timeout-method thread -m gpu > $O/tests_cr.log 2>&1 || { tail -40 $O/tests_cr.log; exit 1; }
tail -1 $O/tests_cr.log
