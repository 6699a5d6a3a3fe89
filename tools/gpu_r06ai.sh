# round 6: elimination builds of the push (wrong physics, timing only):
# without the deposit (PINC_PUSH_SKIP=1) or without the flush (=4), per
# species -- where the electrons' extra time over the ions' goes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
bash tools/gpu_ab.sh r06ai_push_elim base:pinc_amd/lib nodep:pinc_amd/lib_sk1 noflush:pinc_amd/lib_sk4 base2:pinc_amd/lib -- --steps 20 --warmup 3
