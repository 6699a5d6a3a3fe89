set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r05u
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
python3 tools/push_dispatches.py $O/tr > $O/push_dispatches.txt && rm -rf $O/tr
cat $O/push_dispatches.txt | tail -30
bash tools/gpu_r05t.sh || exit 1
