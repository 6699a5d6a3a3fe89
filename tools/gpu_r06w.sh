# round 6: the pair residual norm over 8192 blocks (4 grid-stride steps per
# thread) instead of 2048 (16) -- C4 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
bash tools/gpu_ab.sh r06w_norm_blocks base:pinc_amd/lib nb8:pinc_amd/lib_nb8 base2:pinc_amd/lib nb82:pinc_amd/lib_nb8 -- --steps 20 --warmup 3
