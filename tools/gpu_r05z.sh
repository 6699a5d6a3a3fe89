set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
AB_PMC=1 bash tools/gpu_ab.sh r05z base:pinc_amd/lib xcd:pinc_amd/lib_xcd -- --steps 10 --warmup 3 || exit 1
