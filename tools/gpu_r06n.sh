# round 6: push knob retune after the contiguous streams (XCD piece size,
# LDS charge copies, charge-box size) -- C4 A/B, one run each plus a
# repeat of the base
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
bash tools/gpu_ab.sh r06n_push_knobs base:pinc_amd/lib xp32:pinc_amd/lib_xp32 xp256:pinc_amd/lib_xp256 cp4:pinc_amd/lib_cp4 rl4k:pinc_amd/lib_rl4k base2:pinc_amd/lib -- --steps 30 --warmup 5
