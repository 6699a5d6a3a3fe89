# A/B of in-tree library variants (PINC_LIBDIR, built on the CPU side with
# PINC_LIBDIR=pinc_amd/lib_x PINC_HIP_DEFINES="-D..." python -m pinc_amd.build):
# one bench run per variant under rocprofv3 --kernel-trace --stats, then the
# per-kernel averages side by side (tools/ab_table.py), plus each run's bench
# line.  Optional FETCH_SIZE / WRITE_SIZE passes with AB_PMC=1.
# usage (gpurun): bash tools/gpu_ab.sh <tag> <variant>... [-- bench args]
#   variant = name:libdir[:VAR=value[,VAR=value]]  (environment of that run)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
T=$1; shift
O=gpurun_out/$T
mkdir -p $O
libs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do libs+=("$1"); shift; done
[ "$1" == "--" ] && shift
names=()
for V in "${libs[@]}"; do
  IFS=: read -r n L E <<< "$V"
  names+=("$n")
  envs=(PINC_LIBDIR=$L)
  [ -n "$E" ] && IFS=, read -r -a extra <<< "$E" && envs+=("${extra[@]}")
  env "${envs[@]}" timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$n -o run -- \
    python3 -u bench.py --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 tools/db_stats.py $O/prof_$n $O/${n}_kernel_stats.csv && rm -rf $O/prof_$n
  if [ "${AB_PMC:-0}" == "1" ]; then
    for c in FETCH_SIZE WRITE_SIZE; do
      env "${envs[@]}" timeout -s KILL 300 rocprofv3 --pmc $c -d $O/pmc_${c}_$n -o run -- \
        python3 -u bench.py --no-cpu-baseline --steps 3 --warmup 2 "$@" > /dev/null 2> $O/pmc_${c}_$n.err || { tail -5 $O/pmc_${c}_$n.err; exit 1; }
    done
    python3 tools/pmc_summary.py ${T}_$n $O/pmc_FETCH_SIZE_$n $O/pmc_FETCH_SIZE_$n $O/pmc_WRITE_SIZE_$n $O/$n.json > $O/pmc_$n.txt 2>&1
    rm -rf $O/pmc_FETCH_SIZE_$n $O/pmc_WRITE_SIZE_$n profiles/${T}_${n}_kernel_stats.csv
    mv profiles/${T}_${n}_hbm_traffic.json $O/ 2>/dev/null
  fi
done
python3 tools/ab_table.py $O "${names[@]}" | tee $O/summary.txt
