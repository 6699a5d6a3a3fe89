# round-3 batch d: brick-level counting push A/B against the round-2 kernel,
# then the tiled-layout parity tests on it
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r03d}
mkdir -p gpurun_out/$T
bash tools/gpu_ab.sh ${T}ab base:pinc_amd/lib_base new:pinc_amd/lib -- --steps 40 --warmup 4 > gpurun_out/$T/ab.log 2>&1 || { tail -30 gpurun_out/$T/ab.log; exit 1; }
cat gpurun_out/${T}ab/summary.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_langmuir.py tests/test_gpu_objects.py::test_object_steps_match_checker tests/test_gpu_multirank.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/$T/tests.log 2>&1
rc=$?
tail -5 gpurun_out/$T/tests.log
exit $rc
