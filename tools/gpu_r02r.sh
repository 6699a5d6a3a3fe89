set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02r
mkdir -p $O
for n in 128 256; do
  timeout -k 10 120 python -u tests/mg_history.py --side gpu --size $n --levels 5 --cycles 200 --native --out $O/g${n}_native.json || exit 1
done
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
