# round-end evidence: the default bench line (with cpu_baseline), the C4
# profile passes (kernel stats, FETCH_SIZE, WRITE_SIZE -> profiles/<tag>_*),
# and C3 / C2 / C5 bench lines each under rocprofv3 --kernel-trace --stats.
# usage (gpurun): bash tools/gpu_final.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
T=${1:-final}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench_c4.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 1; }
cat $O/bench_c4.json
bash tools/profile_bench.sh --steps 10 --warmup 3 > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
python3 tools/kernel_gaps.py gpurun_out/prof 12 > $O/${T}_kernel_gaps.txt || exit 1
python3 tools/pmc_summary.py $T gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/prof_bench.json > $O/pmc_summary.txt || exit 1
cp profiles/${T}_* $O/ && cp gpurun_out/prof_bench.json $O/prof_bench_c4.json
rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write
for w in c3 c2 c5 c4ts; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_$w -o run -- python3 bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
  python3 tools/db_stats.py $O/prof_$w $O/${T}_${w}_kernel_stats.csv && rm -rf $O/prof_$w
  python3 -c "
import json; r=json.load(open('$O/bench_$w.json'))
print('$w value %.4g ms/step %.2f solve %.2f' % (r['value'], r['ms_per_step'], r['poisson_ms_per_step']))"
done
