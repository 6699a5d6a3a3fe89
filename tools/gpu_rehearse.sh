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
# eight ranks (the driver's N=8 slab geometry at 256^3, 8 ppc, shard auto; 128^3
# slabs of 16 planes break the reference's trueSize % 2^mgLevels rule) and two
# ranks of C5 (object, replicated solve), both with the extrapolated guesses
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 8 --steps 3 --warmup 2 --size 256 --ppc 8 --host-transport --no-cpu-baseline > $O/bench8.json 2> $O/bench8.err || { tail -30 $O/bench8.err; exit 1; }
python3 -c "
import json; r=json.load(open('$O/bench8.json'))
print('n_gpus', r['n_gpus'], 'value %.4g ms/step %.2f solve %.2f cycles %.2f' % (r['value'], r['ms_per_step'], r['poisson_ms_per_step'], r['mg_cycles_per_solve']), r['config']['poisson'][-90:])"
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 2 --workload c5 --steps 3 --warmup 2 --size 128 --host-transport --no-cpu-baseline > $O/bench2_c5.json 2> $O/bench2_c5.err || { tail -30 $O/bench2_c5.err; exit 1; }
python3 -c "
import json; r=json.load(open('$O/bench2_c5.json'))
print('c5 n_gpus', r['n_gpus'], 'value %.4g ms/step %.2f solve %.2f cycles %.2f' % (r['value'], r['ms_per_step'], r['poisson_ms_per_step'], r['mg_cycles_per_solve']))"
