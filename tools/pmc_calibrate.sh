#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on the GPU box (tools/pmc_calibrate.hip,
# built on the CPU side with
#   hipcc -std=c++17 -O3 --offload-arch=gfx950 -munsafe-fp-atomics tools/pmc_calibrate.hip -o tools/pmc_calibrate)
# usage (gpurun): bash tools/pmc_calibrate.sh <tag>
set -o pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
T=${1:-cal}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 120 ./tools/pmc_calibrate 2048 3 > $O/rates.jsonl || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o cal -- ./tools/pmc_calibrate 2048 1 > /dev/null || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o cal -- ./tools/pmc_calibrate 2048 1 > /dev/null || exit $?
echo "calibration passes done"
