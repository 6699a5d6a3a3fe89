# round 6: LLVM scheduling strategies for every kernel (max-memory-clause,
# max-ilp, occupancy bias 0) -- C4 A/B against the default build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
bash tools/gpu_ab.sh r06ag_sched base:pinc_amd/lib smc:pinc_amd/lib_smc silp:pinc_amd/lib_silp bias:pinc_amd/lib_bias base2:pinc_amd/lib smc2:pinc_amd/lib_smc silp2:pinc_amd/lib_silp -- --steps 20 --warmup 3
