set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r05r
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_errors.py tests/test_c_driver.py tests/test_gpu_scale.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_ab.sh r05r prev:pinc_amd/lib_prev new:pinc_amd/lib -- --steps 10 --warmup 3 || exit 1
for v in prev:pinc_amd/lib_prev new:pinc_amd/lib; do
  n=${v%%:*}; L=${v#*:}
  PINC_LIBDIR=$L timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -d $O/tr_$n -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > /dev/null 2> $O/tr_$n.err || exit 1
  python3 tools/kernel_gaps.py $O/tr_$n 12 > $O/gaps_$n.txt && python3 tools/api_gaps.py $O/tr_$n --step > $O/step_$n.txt && rm -rf $O/tr_$n
done
tail -n 2 $O/gaps_prev.txt $O/gaps_new.txt
