#!/bin/bash
# Round 5 (j): the forced-comm 7B bench again (comm events now recycled only after they complete), then the
# GEMM / fp8 / decode measurements of script g.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5j
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
PADDLE2_AMD_STAGE3_FORCE_COMM=1 timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > $O/bench_force.log 2>&1
r=$?; tail -1 $O/bench_force.log | cut -c1-300; [ $r -ne 0 ] && { grep -v "^\[rank0\]:   " $O/bench_force.log | tail -20; exit $r; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_stage3_force_comm.py tests/test_native_pg_gpu.py tests/test_rccl_gpu.py > $O/tests_comm.log 2>&1
r=$?; tail -2 $O/tests_comm.log; [ $r -ne 0 ] && { grep -E "^E |FAIL" $O/tests_comm.log | head -30; exit $r; }
bash scripts/gpu_r5_g.sh
