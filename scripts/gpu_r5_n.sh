#!/bin/bash
# Round 5 (n): the native allocator no longer returns chunks to the driver mid-run (an OOM settles fences and
# rescans instead).  (1) plain 7B bench with allocator statistics, (2) the forced-comm 7B bench at full batch,
# (3) the comm GPU tests, (4) the GEMM / fp8 / decode measurements of script g.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5n
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
PADDLE2_AMD_BENCH_DEBUG=1 timeout -k 10 400 python -u bench.py --steps 6 --warmup 3 > $O/plain_dbg.log 2>&1
r=$?; echo "plain rc=$r"; grep -E "^\[bench\]|pd_alloc" $O/plain_dbg.log | sort -u; tail -1 $O/plain_dbg.log | cut -c1-200
[ $r -ne 0 ] && { tail -12 $O/plain_dbg.log; exit $r; }
PADDLE2_AMD_BENCH_DEBUG=1 PADDLE2_AMD_STAGE3_FORCE_COMM=1 timeout -k 10 400 python -u bench.py --steps 6 --warmup 5 \
  > $O/force_dbg.log 2>&1
r=$?; echo "force rc=$r"; grep -E "^\[bench\]|pd_alloc" $O/force_dbg.log | sort -u; tail -1 $O/force_dbg.log | cut -c1-200
[ $r -ne 0 ] && { grep -v "^\[rank0\]:   " $O/force_dbg.log | tail -12; exit $r; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_stage3_force_comm.py tests/test_native_pg_gpu.py tests/test_rccl_gpu.py tests/test_native_allocator.py \
  > $O/tests_comm.log 2>&1
r=$?; tail -2 $O/tests_comm.log; [ $r -ne 0 ] && { grep -E "^E |FAIL" $O/tests_comm.log | head -30; exit $r; }
bash scripts/gpu_r5_g.sh
