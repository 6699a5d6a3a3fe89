set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05l
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reference_kat.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/r05l/tests.log 2>&1 || { tail -30 gpurun_out/r05l/tests.log; exit 1; }
tail -2 gpurun_out/r05l/tests.log
bash tools/gpu_ab.sh r05l prev:pinc_amd/lib_prev new:pinc_amd/lib -- --steps 10 --warmup 3
PINC_LIBDIR=pinc_amd/lib timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --kernel-include-regex "k_push" -d gpurun_out/r05l/pmc_new -o push -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2>&1 && python3 tools/pmc_dispatches.py gpurun_out/r05l/pmc_new k_push gpurun_out/r05l/pmc_new.csv && rm -rf gpurun_out/r05l/pmc_new
