# round 6: cell-ranked sorting push as the default -- C4 A/B at the
# bench's default 50 steps against the previous library, then the full GPU
# suite and smoke, then the round-end evidence (tools/gpu_final.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
bash tools/gpu_ab.sh r06al_cellrank_default old:pinc_amd/lib_old new:pinc_amd/lib old2:pinc_amd/lib_old new2:pinc_amd/lib || exit 1
bash tools/gpu_r06suite.sh r06al || exit 1
bash tools/gpu_final.sh r06zzzz || exit 1
