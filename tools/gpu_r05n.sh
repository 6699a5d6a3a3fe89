set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05n
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reference_kat.py tests/test_gpu_multirank.py tests/test_gpu_objects.py tests/test_gpu_langmuir.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/r05n/tests.log 2>&1 || { tail -30 gpurun_out/r05n/tests.log; exit 1; }
tail -2 gpurun_out/r05n/tests.log
bash tools/gpu_ab.sh r05n noskip:pinc_amd/lib:PINC_EXTRACT_SKIP=0 skip:pinc_amd/lib -- --steps 10 --warmup 3
for v in 0 1; do
  PINC_EXTRACT_SKIP=$v timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r05n/gaps_$v -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > /dev/null 2> gpurun_out/r05n/gaps_$v.err || exit 1
  python3 tools/kernel_gaps.py gpurun_out/r05n/gaps_$v 12 > gpurun_out/r05n/gaps_$v.txt && rm -rf gpurun_out/r05n/gaps_$v
done
tail -3 gpurun_out/r05n/gaps_0.txt gpurun_out/r05n/gaps_1.txt
