# LDS / issue counters of the multigrid kernels (rep256 probe).  usage (gpurun): bash tools/gpu_mgpmc2.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1 PMC_MIN_GRID=65536
O=gpurun_out/${1:-mgpmc2}
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
	-d $O/pmcA -o run -- python3 tools/mg_shard_probe.py --cases rep256 --out $O/a.json > $O/pmcA.log 2>&1 &&
python3 tools/pmc_kernels.py $O/pmcA $O/pmcA_summary.json > /dev/null && rm -rf $O/pmcA &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM \
	-d $O/pmcB -o run -- python3 tools/mg_shard_probe.py --cases rep256 --out $O/b.json > $O/pmcB.log 2>&1 &&
python3 tools/pmc_kernels.py $O/pmcB $O/pmcB_summary.json > /dev/null && rm -rf $O/pmcB
