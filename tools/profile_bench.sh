#!/bin/bash
# Profile the default bench command on the GPU box (run through gpurun):
#   1. rocprofv3 --kernel-trace --stats  -> gpurun_out/prof/bench_kernel_stats.csv
#   2. --pmc FETCH_SIZE and 3. --pmc WRITE_SIZE in passes of their own
#      (MI355X_MICROARCH.md: the two do not fit one TCC pass)
# then summarise with tools/pmc_summary.py <tag> into profiles/.
# Extra arguments are passed to bench.py in every pass.
set -o pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench -- \
	python3 bench.py --no-cpu-baseline "$@" > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err || exit $?
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o bench -- \
	python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/pmc_fetch.json 2> gpurun_out/pmc_fetch.err || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o bench -- \
	python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/pmc_write.json 2> gpurun_out/pmc_write.err || exit $?
echo "profile passes done"
