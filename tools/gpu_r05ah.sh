set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r05ah
mkdir -p $O
PINC_LIBDIR=pinc_amd/lib_cr timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_multirank.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_ab.sh r05ah base:pinc_amd/lib cr:pinc_amd/lib_cr -- --steps 30 --warmup 3 || exit 1
PINC_LIBDIR=pinc_amd/lib_cr timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > /dev/null 2> $O/tr.err || exit 1
python3 tools/push_dispatches.py $O/tr > $O/push_dispatches_cr.txt && rm -rf $O/tr
