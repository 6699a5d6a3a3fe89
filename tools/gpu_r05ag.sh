set -o pipefail
cd $GRAFT_REPO_ROOT
export PINC_QUIET=1
bash tools/pmc_push.sh r05ag --steps 9 --warmup 1 > gpurun_out/r05ag_pmc.log 2>&1 || { tail -20 gpurun_out/r05ag_pmc.log; exit 1; }
ls gpurun_out/r05ag
