# round-3 batch: FETCH/WRITE calibration, the new scale / pairing / MG
# fixture / sharded-object / graph-replay tests, then the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r03b}
bash tools/pmc_calibrate.sh ${T}cal > gpurun_out/${T}cal.log 2>&1 || exit 1
mkdir -p gpurun_out/$T
timeout -k 10 1000 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_comm_pairing.py tests/test_gpu_mg_scale.py "tests/test_gpu_objects.py::test_object_two_slabs_match_one" "tests/test_gpu_parity.py::test_native_mg_graph_replay" -v -s --timeout 400 --timeout-method thread -m gpu --durations=40 > gpurun_out/$T/tests.log 2>&1
rc=$?
tail -45 gpurun_out/$T/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/$T/bench_c4.json 2> gpurun_out/$T/bench_c4.err || { tail -20 gpurun_out/$T/bench_c4.err; exit 1; }
cat gpurun_out/$T/bench_c4.json
