# push experiment: parity tests of the push with the default library, then
# a short bench per library variant.  usage (gpurun): bash tools/gpu_pushvar.sh <tag> <libdir>...
set -o pipefail
cd $GRAFT_REPO_ROOT
export PINC_QUIET=1
T=$1; shift
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py tests/test_gpu_errors.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_variants.sh $T "$@"
