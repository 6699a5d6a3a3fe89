# run a set of GPU test files; usage (gpurun): bash tools/gpu_tests.sh <tag> <test files...>
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-tests}; shift
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1
rc=$?
tail -30 $O/tests.log
exit $rc
