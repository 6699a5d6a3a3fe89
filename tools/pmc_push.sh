#!/bin/bash
# Instruction-mix PMC passes of the push (k_push) at C4 on the GPU box:
# three passes of at most 8 SQ counters each (MI355X_MICROARCH.md: one pass
# cannot split counters), each a short bench run, then per-dispatch CSVs
# (tools/pmc_dispatches.py).  usage (gpurun): bash tools/pmc_push.sh <tag> [bench args]
set -o pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
T=${1:-pmcpush}; shift
O=gpurun_out/$T
mkdir -p $O
P=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVE_CYCLES"
  "SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INST_CYCLES_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
  "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64 SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT"
)
i=0
for c in "${P[@]}"; do
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-include-regex "k_push" -d $O/p$i -o push -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > $O/p$i.json 2> $O/p$i.err || exit $?
  python3 tools/pmc_dispatches.py $O/p$i k_push $O/p$i.csv || exit $?
  i=$((i+1))
done
echo "pmc push passes done"
