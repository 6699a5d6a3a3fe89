# round 6: the sorting push ranks each thread's same-brick items as one run
# (PINC_PUSH_SORT_RUNS) -- parity tests with sorting pushes, then an A/B
# against per-item ranking (lib_sr0); 50 steps so several sort cycles land
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r06h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_flag_switches.py -x -v --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
bash tools/gpu_ab.sh r06h_sortruns sr0:pinc_amd/lib_sr0 runs:pinc_amd/lib sr0b:pinc_amd/lib_sr0 runsb:pinc_amd/lib -- --steps 50 --warmup 5
