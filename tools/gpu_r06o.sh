# round 6: the level-0 double sweep on 64x8 tiles of 512 threads
# (PINC_MG_S4_WIDE, lib_sw) -- its bit-identity tests, then a C4 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r06o
mkdir -p $O
PINC_LIBDIR=pinc_amd/lib_sw timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mg_sine.py -x -v --timeout 200 --timeout-method thread -m gpu > $O/tests_sw.log 2>&1 || { tail -40 $O/tests_sw.log; exit 1; }
tail -1 $O/tests_sw.log
bash tools/gpu_ab.sh r06o_sweep_wide base:pinc_amd/lib wide:pinc_amd/lib_sw base2:pinc_amd/lib wide2:pinc_amd/lib_sw -- --steps 20 --warmup 3
