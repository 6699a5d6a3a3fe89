# round 6: the one-workgroup small solve -- the full GPU suite, smoke, and
# C2 A/B (one workgroup against the per-level graph path)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r06m2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
bash tools/gpu_ab.sh r06m2_c2 graph:pinc_amd/lib:PINC_MG_SMALL=0 onecu:pinc_amd/lib graph2:pinc_amd/lib:PINC_MG_SMALL=0 onecu2:pinc_amd/lib -- --workload c2 --steps 200 --warmup 20
