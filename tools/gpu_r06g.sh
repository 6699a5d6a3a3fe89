# round 6: nontemporal particle loads/stores on the push's contiguous path
# (PINC_PUSH_XCH_NT 1 loads, 2 stores, 3 both) against plain (lib)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
bash tools/gpu_ab.sh r06g_nt base:pinc_amd/lib nt1:pinc_amd/lib_nt1 nt2:pinc_amd/lib_nt2 nt3:pinc_amd/lib_nt3 base2:pinc_amd/lib -- --steps 30 --warmup 3
