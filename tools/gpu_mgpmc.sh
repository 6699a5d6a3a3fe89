# SQ counters of the multigrid kernels (rep256 solve of tools/mg_shard_probe.py)
# usage (gpurun): bash tools/gpu_mgpmc.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1 PMC_MIN_GRID=65536
O=gpurun_out/${1:-mgpmc}
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- python3 tools/mg_shard_probe.py --cases rep256 --out $O/kt.json > $O/kt.log 2>&1 &&
python3 -c "
import sqlite3,glob
db=sqlite3.connect(glob.glob(\"$O/kt/**/*.db\",recursive=True)[0])
for r in db.execute(\"select * from top_kernels limit 12\"): print(r)
" > $O/kt_top.txt && rm -rf $O/kt &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
	-d $O/pmcA -o run -- python3 tools/mg_shard_probe.py --cases rep256 --out $O/a.json > $O/pmcA.log 2>&1 &&
python3 tools/pmc_kernels.py $O/pmcA $O/pmcA_summary.json > /dev/null &&
rm -rf $O/pmcA &&
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_RD \
	-d $O/pmcB -o run -- python3 tools/mg_shard_probe.py --cases rep256 --out $O/b.json > $O/pmcB.log 2>&1 &&
python3 tools/pmc_kernels.py $O/pmcB $O/pmcB_summary.json > /dev/null &&
rm -rf $O/pmcB &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmcF -o run -- python3 tools/mg_shard_probe.py --cases rep256 --out $O/f.json > $O/pmcF.log 2>&1 &&
python3 tools/pmc_kernels.py $O/pmcF $O/pmcF_summary.json > /dev/null &&
rm -rf $O/pmcF &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmcW -o run -- python3 tools/mg_shard_probe.py --cases rep256 --out $O/w.json > $O/pmcW.log 2>&1 &&
python3 tools/pmc_kernels.py $O/pmcW $O/pmcW_summary.json > /dev/null &&
rm -rf $O/pmcW
