# round 6: the full GPU suite and smoke on the current tree (tag as $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r06suite}
mkdir -p gpurun_out/$T
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/$T/gpu_full_suite.log 2>&1 || { tail -30 gpurun_out/$T/gpu_full_suite.log; exit 1; }
tail -1 gpurun_out/$T/gpu_full_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$T/smoke.log 2>&1 || { tail -20 gpurun_out/$T/smoke.log; exit 1; }
tail -1 gpurun_out/$T/smoke.log
