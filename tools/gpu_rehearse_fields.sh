# The N>1 bench line's diagnostic fields at the driver's geometry: N ranks
# share one GPU over the host transport (gloo), 256^3 with 8 ppc per species
# (the grid-sized exchanges -- folds, halos, gathers, reductions -- are the
# full-size ones; migration bytes scale with ppc), C4 at N = 2, 4, 8 and C5
# (sharded objects) at N = 4.  Times are not RCCL times (gloo, one shared
# GPU); bytes and calls per step are what an 8-GPU run moves.
# usage (gpurun): bash tools/gpu_rehearse_fields.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export PINC_QUIET=1
O=gpurun_out/${1:-rehearse_fields}
mkdir -p $O
port=29541
for spec in c4:2 c4:4 c4:8 c5:4; do
  IFS=: read -r w n <<< "$spec"
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus $n --workload $w --steps 3 --warmup 2 --size 256 --ppc 8 --host-transport \
    --no-cpu-baseline > $O/${w}_n$n.json 2> $O/${w}_n$n.err || { tail -30 $O/${w}_n$n.err; exit 1; }
  port=$((port + 1))
  python3 tools/multi_rank_table.py $O/${w}_n$n.json
done
