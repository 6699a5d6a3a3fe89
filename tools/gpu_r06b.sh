# round 6: sparse flag writes and the decomposed level 1 -- the parity tests
# that touch flags, the extraction and the sharded multigrid; the copy
# ceilings of k_push's lane mapping; an A/B of PINC_FLAGS_SPARSE 0/1
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r06b
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/test_gpu_flag_switches.py tests/test_gpu_mg_shard.py tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_errors.py tests/test_gpu_objects.py tests/test_gpu_mg_sine.py -x -v --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for w in 24 8; do
  timeout -k 10 120 tools/copy_probe3 8192 3 $w >> $O/copy_probe3.jsonl 2>&1 || { tail -5 $O/copy_probe3.jsonl; exit 1; }
done
cat $O/copy_probe3.jsonl
AB_PMC=1 bash tools/gpu_ab.sh r06b_flags full:pinc_amd/lib:PINC_FLAGS_SPARSE=0 sparse:pinc_amd/lib:PINC_FLAGS_SPARSE=1 -- --steps 30 --warmup 3
