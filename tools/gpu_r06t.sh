# round 6: the push at three waves per SIMD (PINC_PUSH_WPE=3: 135 VGPRs
# instead of 121 at four) -- C4 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
bash tools/gpu_ab.sh r06t_push_wpe3 base:pinc_amd/lib w3:pinc_amd/lib_w3 base2:pinc_amd/lib w32:pinc_amd/lib_w3 -- --steps 20 --warmup 3
