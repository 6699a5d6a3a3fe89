# round 6: push blocks of 512 threads (2048 particles, 8 waves; E box 1536
# nodes, charge LDS 4096 doubles: two blocks per CU at four waves per SIMD)
# -- C4 A/B against the default 256-thread blocks, two runs each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
bash tools/gpu_ab.sh r06ac_push_512 base:pinc_amd/lib t512:pinc_amd/lib_t512 base2:pinc_amd/lib t512b:pinc_amd/lib_t512 -- --steps 20 --warmup 3
