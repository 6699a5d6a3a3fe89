# round 6: the level-0 double sweep gathering rho from a colour-split copy
# (no rho ring, 40 KB of LDS, three workgroups per CU; lib_rs) -- its
# bit-identity and multigrid tests, then a C4 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r06r
mkdir -p $O
PINC_LIBDIR=pinc_amd/lib_rs timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mg_sine.py tests/test_gpu_mg_scale.py -x -v --timeout 300 --timeout-method thread -m gpu > $O/tests_rs.log 2>&1 || { tail -40 $O/tests_rs.log; exit 1; }
tail -1 $O/tests_rs.log
bash tools/gpu_ab.sh r06r_sweep_rho_split base:pinc_amd/lib rs:pinc_amd/lib_rs base2:pinc_amd/lib rs2:pinc_amd/lib_rs -- --steps 20 --warmup 3
