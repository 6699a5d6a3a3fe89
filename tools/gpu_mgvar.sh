# multigrid kernel experiment: the sweep kernel tests, then the rep256 probe
# with each library variant.  usage (gpurun): bash tools/gpu_mgvar.sh <tag> <libdir>...
set -o pipefail
cd $GRAFT_REPO_ROOT
export PINC_QUIET=1
T=$1; shift
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -m gpu -k sweep > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for L in "$@"; do
  n=$(basename $L)
  PINC_LIBDIR=$L timeout -k 10 200 python -u tools/mg_shard_probe.py --cases rep256,rep_l1 --out $O/$n.json > $O/$n.log 2>&1 || exit 1
  echo "$n: $(grep -o '"case": "[a-z0-9_]*"\|"ms_per_cycle": [0-9.]*' $O/$n.log | tr '\n' ' ')"
done
