# round 6: the level-0 double sweep without the rho ring (rho gathered per
# stage, 40 KB of LDS: three workgroups per CU at 143 VGPRs; lib_r0) --
# its bit-identity tests, then a C4 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r06q
mkdir -p $O
PINC_LIBDIR=pinc_amd/lib_r0 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 200 --timeout-method thread -m gpu -k "sweep" > $O/tests_r0.log 2>&1 || { tail -40 $O/tests_r0.log; exit 1; }
tail -1 $O/tests_r0.log
bash tools/gpu_ab.sh r06q_sweep_noring base:pinc_amd/lib r0:pinc_amd/lib_r0 base2:pinc_amd/lib r02:pinc_amd/lib_r0 -- --steps 20 --warmup 3
