# round-5 final tree: full GPU suite, smoke, then the evidence run (bench
# lines, rocprof stats, PMC passes, kernel gaps) under the tag r05zzzfinal
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05zzzfinal
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r05zzzfinal/gpu_full_suite.log 2>&1 || { tail -30 gpurun_out/r05zzzfinal/gpu_full_suite.log; exit 1; }
tail -1 gpurun_out/r05zzzfinal/gpu_full_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05zzzfinal/smoke.log 2>&1 || { tail -20 gpurun_out/r05zzzfinal/smoke.log; exit 1; }
tail -1 gpurun_out/r05zzzfinal/smoke.log
bash tools/gpu_final.sh r05zzzfinal
