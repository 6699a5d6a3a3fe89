# E chain in the push: parity tests, then an A/B of the C4 bench (the push
# gathering from E with the species chain vs the k_field_chain copy)
set -o pipefail
O=gpurun_out/r05t
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_reference_kat.py tests/test_gpu_scale.py tests/test_gpu_mg_sine.py tests/test_gpu_mg_scale.py -k "not full_size" > $O/tests.log 2>&1 || exit $?
for v in 1 0 1 0; do
  PINC_PUSH_ECHAIN=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c4_$v.json 2>$O/c4_$v.log || exit $?
  python tools/bench_line.py $O/c4_$v.json
done
