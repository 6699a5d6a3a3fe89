set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r05o
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -d $O/tr -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 tools/api_gaps.py $O/tr 20 10 > $O/api_gaps.txt 2>&1
python3 tools/kernel_gaps.py $O/tr 12 > $O/gaps.txt 2>&1
rm -rf $O/tr
cat $O/api_gaps.txt | head -80
