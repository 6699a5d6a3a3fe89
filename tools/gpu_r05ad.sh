set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ad
mkdir -p $O
PINC_LIBDIR=pinc_amd/lib_nobox timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q --timeout 200 --timeout-method thread -m gpu -k "graph_replay" > $O/nobox.log 2>&1; echo "nobox rc=$?"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q --timeout 200 --timeout-method thread -m gpu -k "graph_replay" > $O/box.log 2>&1; echo "box rc=$?"
tail -3 $O/nobox.log $O/box.log
