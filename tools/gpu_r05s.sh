set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r05s
mkdir -p $O
AB_PMC=1 bash tools/gpu_ab.sh r05s base:pinc_amd/lib s4:pinc_amd/lib_s4 s2:pinc_amd/lib_s2 -- --steps 10 --warmup 3 || exit 1
PINC_TRACE_SORT=2 timeout -k 10 300 python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline > $O/trace.json 2> $O/trace.err || exit 1
grep "push species" $O/trace.err > $O/push_phases.txt
timeout -k 10 120 rocprofv3 --list-avail > $O/counters.txt 2>&1 || true
grep -i -E "icache|ifetch|SQC_" $O/counters.txt | head -40 > $O/counters_sqc.txt || true
timeout -s KILL 90 rocprofv3 --pmc SQ_IFETCH SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-include-regex "k_push" -d $O/pmc_if -o push -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $O/pmc_if.err && python3 tools/pmc_dispatches.py $O/pmc_if k_push $O/pmc_if.csv && rm -rf $O/pmc_if
echo done
