set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r05k
mkdir -p $O
for v in lib lib_skip1 lib_skip2 lib_skip4; do
  PINC_LIBDIR=pinc_amd/$v timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-include-regex "k_push" -d $O/$v -o push -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/$v.json 2> $O/$v.err || exit $?
  python3 tools/pmc_dispatches.py $O/$v k_push $O/$v.csv || exit $?
  rm -rf $O/$v
done
echo done
