# round 6: kernel arguments in device memory or host memory
# (HIP_FORCE_DEV_KERNARG=1 / 0) -- C4 A/B against the runtime's default
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
bash tools/gpu_ab.sh r06ah_kernarg base:pinc_amd/lib dev:pinc_amd/lib:HIP_FORCE_DEV_KERNARG=1 host:pinc_amd/lib:HIP_FORCE_DEV_KERNARG=0 base2:pinc_amd/lib dev2:pinc_amd/lib:HIP_FORCE_DEV_KERNARG=1 -- --steps 20 --warmup 3
