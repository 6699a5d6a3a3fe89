# parity tests of the push, then the three profile passes of the default
# bench command (kernel trace + stats, FETCH_SIZE, WRITE_SIZE), summarised
# into profiles/<tag>_*.  usage (gpurun): bash tools/gpu_profile.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-prof}
export TMPDIR=/tmp
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/$T/tests.log 2>&1 || exit 1
bash tools/profile_bench.sh --steps 10 --warmup 3 || exit 1
python3 tools/pmc_summary.py $T gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write > gpurun_out/$T/pmc_summary.txt || exit 1
cp profiles/${T}_* gpurun_out/$T/
cp gpurun_out/prof_bench.json gpurun_out/$T/prof_bench.json
rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write
