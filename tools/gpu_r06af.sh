# round 6: the push rescales the E values it reads (species chain, no stored
# rescaled copy, no k_field_chain_all pass) -- C4 A/B against the previous
# library; "nochain" is the new library with PINC_PUSH_ECHAIN=0
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
bash tools/gpu_ab.sh r06af_push_echain old:pinc_amd/lib_old new:pinc_amd/lib nochain:pinc_amd/lib:PINC_PUSH_ECHAIN=0 old2:pinc_amd/lib_old new2:pinc_amd/lib -- --steps 20 --warmup 3
