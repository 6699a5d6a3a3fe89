# push sort experiment: GPU tests ($TESTS) with the default library, then per
# library variant a steady-state bench line (40 timed steps after 12 warm-up
# steps) and a phase trace (mean span per push kind).
# usage (gpurun): bash tools/gpu_sortab.sh <tag> <libdir>...
set -o pipefail
cd $GRAFT_REPO_ROOT
export PINC_QUIET=1
T=$1; shift
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_kernels.py tests/test_gpu_objects.py tests/test_gpu_multirank.py tests/test_gpu_errors.py} -x -q --timeout 200 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for L in "$@"; do
  n=$(basename $L)
  PINC_LIBDIR=$L timeout -k 10 300 python -u bench.py --steps 40 --warmup 12 --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
  PINC_LIBDIR=$L PINC_TRACE_SORT=2 timeout -k 10 300 python -u bench.py --steps 24 --warmup 2 --no-cpu-baseline > $O/$n.trace.json 2> $O/$n.trace.err || { tail -5 $O/$n.trace.err; exit 1; }
  grep "push species" $O/$n.trace.err > $O/$n.push_trace.txt || true
  python3 - "$O" "$n" <<'PY' | tee -a $O/summary.txt
import json, re, sys, collections
O, n = sys.argv[1], sys.argv[2]
r = json.load(open(f"{O}/{n}.json")); k = r["kernels"]
sp = collections.defaultdict(list)
for l in open(f"{O}/{n}.push_trace.txt"):
    m = re.search(r"species (\d)( sort)?( count)?: span ([\d.]+)", l)
    if m: sp[(m.group(1), (m.group(2) or m.group(3) or " plain").strip())].append(float(m.group(4)))
kinds = " ".join(f"s{s}-{t} {sum(v)/len(v):.1f}x{len(v)}" for (s, t), v in sorted(sp.items()))
print("%-12s value %.4g ms/step %.2f solve %.2f push %.3f ms frac %.3f | %s" % (n, r["value"], r["ms_per_step"], r["poisson_ms_per_step"], k["push"]["mean_launch_ms"], k["push"]["frac"], kinds))
PY
done
