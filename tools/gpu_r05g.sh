set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r05g.log 2>&1 || { tail -20 gpurun_out/smoke_r05g.log; exit 1; }
tail -1 gpurun_out/smoke_r05g.log
bash tools/gpu_final.sh r05g
