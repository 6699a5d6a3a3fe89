set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ae
mkdir -p $O
PINC_LIBDIR=pinc_amd/lib_bc timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -s --timeout 200 --timeout-method thread -m gpu -k "graph_replay and c2" > $O/bc.log 2>&1; echo "bc rc=$?"
grep -c boxcheck $O/bc.log; grep boxcheck $O/bc.log | head -20
