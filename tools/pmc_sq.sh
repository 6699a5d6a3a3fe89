#!/bin/bash
# One rocprofv3 --pmc pass of SQ counters over a short bench run (kernel
# mix: instruction counts and wait cycles per kernel).  Usage (gpurun):
#   bash tools/pmc_sq.sh <outdir> [bench args]
set -o pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
out=${1:-gpurun_out/pmc_sq}; shift
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
	-d "$out" -o bench -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > "$out.json" 2> "$out.err"
