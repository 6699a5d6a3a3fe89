# round 6: wave priority (s_setprio 1 or 3) for the push's particle-load
# phase -- C4 A/B against the default (no priority change)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
bash tools/gpu_ab.sh r06ad_push_prio base:pinc_amd/lib pr1:pinc_amd/lib_pr1 pr3:pinc_amd/lib_pr3 base2:pinc_amd/lib pr1b:pinc_amd/lib_pr1 pr3b:pinc_amd/lib_pr3 -- --steps 20 --warmup 3
