set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r06y2
timeout -k 10 200 python -u -m pytest "tests/test_gpu_parity.py::test_native_mg_graph_replay" -x -v -s --timeout 120 --timeout-method thread -m gpu > gpurun_out/r06y2/t.log 2>&1; echo "rc=$?" >> gpurun_out/r06y2/t.log
tail -30 gpurun_out/r06y2/t.log
