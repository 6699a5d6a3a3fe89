# four-rank rehearsals on one GPU over the host transport: the sharded-MG
# parity test and the bench's multi-rank flow with the shard forced.
# usage (gpurun): bash tools/gpu_rehearse.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export PINC_QUIET=1
O=gpurun_out/${1:-rehearse}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_mg_shard.py -x -v --timeout 400 --timeout-method thread -m gpu -k "four or two_ranks" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -4 $O/tests.log
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --steps 3 --warmup 1 --size 128 --host-transport --mg-shard 1 --no-cpu-baseline > $O/bench4.json 2> $O/bench4.err || { tail -30 $O/bench4.err; exit 1; }
python3 -c "
import json; r=json.load(open('$O/bench4.json'))
print('n_gpus', r['n_gpus'], 'value %.4g ms/step %.2f solve %.2f' % (r['value'], r['ms_per_step'], r['poisson_ms_per_step']), r['config']['poisson'][-90:])"
