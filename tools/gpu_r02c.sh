set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r02c}
mkdir -p $O
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
	-d $O/pmcA -o bench -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmcA.json 2> $O/pmcA.err &&
python3 tools/pmc_kernels.py $O/pmcA $O/pmcA_summary.json > /dev/null &&
rm -rf $O/pmcA &&
timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_RD \
	-d $O/pmcB -o bench -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmcB.json 2> $O/pmcB.err &&
python3 tools/pmc_kernels.py $O/pmcB $O/pmcB_summary.json > /dev/null &&
rm -rf $O/pmcB
