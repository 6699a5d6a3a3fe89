# round-3 batch c: push-variant A/B (buffer streams, deferred global E
# gather, velocity output buffer), MG XCD tile order, calibration v3, then
# the GPU suite on the default library and the parity file with the
# velocity output buffer on
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r03c}
mkdir -p gpurun_out/$T
bash tools/pmc_calibrate.sh ${T}cal > gpurun_out/${T}cal.log 2>&1 || exit 1
bash tools/gpu_ab.sh ${T}ab base:pinc_amd/lib_base new:pinc_amd/lib newvout:pinc_amd/lib:PINC_PUSH_VOUT=1 nobuf:pinc_amd/lib_nobuf mgxcd:pinc_amd/lib_mgxcd -- --steps 24 --warmup 4 > gpurun_out/$T/ab.log 2>&1 || { tail -30 gpurun_out/$T/ab.log; exit 1; }
cat gpurun_out/${T}ab/summary.txt
PINC_PUSH_VOUT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_errors.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/$T/vout_tests.log 2>&1 || { tail -30 gpurun_out/$T/vout_tests.log; exit 1; }
tail -3 gpurun_out/$T/vout_tests.log
timeout -k 10 1000 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu --durations=30 > gpurun_out/$T/tests.log 2>&1
rc=$?
tail -40 gpurun_out/$T/tests.log
exit $rc
