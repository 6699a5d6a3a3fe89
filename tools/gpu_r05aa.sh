set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r05aa
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu -k "step or energy or history" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 1 0; do
  PINC_BENCH_PYLOOP=$v timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr_$v -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || exit 1
  python3 tools/kernel_gaps.py $O/tr_$v 12 > $O/gaps_$v.txt && rm -rf $O/tr_$v
  python3 -c "import json; r=json.load(open('$O/bench_$v.json')); print('pyloop=$v', r['value'], r['ms_per_step'])"
done
tail -n 1 $O/gaps_1.txt $O/gaps_0.txt
