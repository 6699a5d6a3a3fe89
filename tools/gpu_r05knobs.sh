# push knob re-check on the round-5 push: deposit group minimum (4, 10
# against 6), charge-box copies (4 against 8), XCD piece (128 against 64)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_ab.sh r05knobs base:pinc_amd/lib gm4:pinc_amd/lib_kgm4 gm10:pinc_amd/lib_kgm10 cp4:pinc_amd/lib_kcp4 xp128:pinc_amd/lib_kxp128 base2:pinc_amd/lib -- --steps 10 --warmup 3
