# round 6: the C4 solve's per-cycle residuals (PINC_VERBOSE=1) and a
# smoothing sweep around 4/4; then the N-rank bench fields with level 1
# decomposed (host-transport rehearsal at the driver's geometry)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r06f
mkdir -p $O
PINC_VERBOSE=1 timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 --no-cpu-baseline > $O/verbose.json 2> $O/verbose.err || { tail -20 $O/verbose.err; exit 1; }
grep "solve cycle" $O/verbose.err | tail -40
OUT=$O/smooth STEPS=20 VARIANTS="4,4 5,3 3,5 5,5 5,4 4,5 6,4" bash tools/mg_smooth_sweep.sh || exit 1
bash tools/gpu_rehearse_fields.sh r06f_rehearse || exit 1
