set -o pipefail
mkdir -p gpurun_out/r05s
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_scale.py tests/test_gpu_mg_sine.py "tests/test_gpu_parity.py::test_native_mg_graph_replay" tests/test_gpu_objects.py -k "not full_size or c4" > gpurun_out/r05s/tests.log 2>&1 || exit $?
for v in "4,4" "ini"; do
  timeout -k 10 200 python -u bench.py --workload c2 --steps 10 --warmup 3 --no-cpu-baseline --mg-smooth $v > gpurun_out/r05s/c2_$v.json 2>gpurun_out/r05s/c2_$v.log || exit $?
done
