# kernel statistics of the sharded / replicated solves and one bench line
# with the migration volume.  usage (gpurun): bash tools/gpu_shardprof.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
T=${1:-shardprof}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/ext80 -o run -- python3 tools/mg_shard_probe.py --cases ext80 --out $O/ext80.json > $O/ext80.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/rep256 -o run -- python3 tools/mg_shard_probe.py --cases rep256 --out $O/rep256.json > $O/rep256.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err &&
find $O -name "*kernel_stats.csv" | head
