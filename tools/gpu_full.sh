# the whole -m gpu suite, then smoke().  usage (gpurun): bash tools/gpu_full.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-full}
mkdir -p $O
export PINC_QUIET=1
timeout -k 10 1000 python -u -m pytest tests/ -x -v --timeout 300 --timeout-method thread -m gpu > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
