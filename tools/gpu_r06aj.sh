# round 6: the deposit keeps two open charge runs per thread
# (PINC_PUSH_RUN2=1) -- C4 A/B against the default, two runs each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
bash tools/gpu_ab.sh r06aj_push_run2 base:pinc_amd/lib run2:pinc_amd/lib_r2 base2:pinc_amd/lib run2b:pinc_amd/lib_r2 -- --steps 20 --warmup 3
