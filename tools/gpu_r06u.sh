# round 6: E = -grad phi by slab planes (32-bit coordinates) and the
# species' field chain on 16-B pairs with nontemporal stores -- the step and
# Langmuir parity tests, then a C4 A/B against the previous library
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PINC_QUIET=1
O=gpurun_out/r06u
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_langmuir.py tests/test_gpu_scale.py tests/test_gpu_reference_kat.py -x -v --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab.sh r06u_efield_chain old:pinc_amd/lib_old new:pinc_amd/lib old2:pinc_amd/lib_old new2:pinc_amd/lib -- --steps 20 --warmup 3
