set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02b
timeout -k 10 900 python -u -m pytest tests/ -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/r02b/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02b/smoke.log 2>&1
