# round 6: a fifth wave per SIMD for the push (PINC_PUSH_WPE=5, 96 VGPRs
# with spills) with smaller LDS boxes (E box 512 nodes, charge box 1024),
# and the smaller boxes alone at four waves -- C4 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
bash tools/gpu_ab.sh r06x_push_five_waves base:pinc_amd/lib o5:pinc_amd/lib_o5 sb:pinc_amd/lib_sb base2:pinc_amd/lib -- --steps 20 --warmup 3
