set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02a
export PINC_VERBOSE=250
timeout -k 10 300 python -u tests/mg_history.py --side gpu --size 128 --levels 5 --cycles 3000 --out gpurun_out/r02a/g128.json --phi-out gpurun_out/r02a/g128_phi.npy &&
timeout -k 10 400 python -u tests/mg_history.py --side gpu --size 256 --levels 5 --cycles 3000 --out gpurun_out/r02a/g256.json --phi-out gpurun_out/r02a/g256_phi.npy --phi-stride 2 &&
unset PINC_VERBOSE &&
timeout -k 10 600 python -u -m pytest tests/test_c_driver.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/r02a/cdriver.log 2>&1
