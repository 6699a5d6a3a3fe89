# round 6: copy ceilings of k_push's lane mapping (tools/copy_probe3.hip),
# then the sharded multigrid with level 1 decomposed (tests)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r06c
mkdir -p $O
for w in 24 8; do
  timeout -k 10 120 tools/copy_probe3 8192 3 $w >> $O/copy_probe3.jsonl 2>&1 || { tail -5 $O/copy_probe3.jsonl; exit 1; }
done
cat $O/copy_probe3.jsonl
timeout -k 10 900 python -u -m pytest tests/test_gpu_mg_shard.py tests/test_gpu_mg_sine.py "tests/test_gpu_multirank.py::test_two_ranks_one_gpu" tests/test_gpu_objects.py -x -v --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
