# round 6: wave priority 1 or 3 for everything after the push's particle
# loads (the loads at priority 0) -- C4 A/B against the default
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
bash tools/gpu_ab.sh r06ae_push_prio_rest base:pinc_amd/lib pm1:pinc_amd/lib_pm1 pm3:pinc_amd/lib_pm3 base2:pinc_amd/lib pm1b:pinc_amd/lib_pm1 pm3b:pinc_amd/lib_pm3 -- --steps 20 --warmup 3
