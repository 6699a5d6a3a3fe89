set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
bash tools/gpu_ab.sh r05t base:pinc_amd/lib tw8:pinc_amd/lib:PINC_TILE_WIDTH=8 tw2:pinc_amd/lib:PINC_TILE_WIDTH=2 dk:pinc_amd/lib_dk -- --steps 10 --warmup 3 || exit 1
