#!/bin/bash
# GEMM GPU tests (v2 descriptors now bounded), then the 7B bench on the native allocator with no guard bytes
# and the allocation trace on (a fault leaves the live-block map for scripts/alloc_fault_map.py)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemm_gpu.py \
    > gpurun_out/gemm_tests_r3.log 2>&1
rc=$?; tail -3 gpurun_out/gemm_tests_r3.log; [ $rc -eq 0 ] || exit $rc
FLAGS_use_native_allocator=1 PD_ALLOC_TRACE=gpurun_out/alloc_trace.txt timeout -k 10 400 \
    python -u bench.py --steps 4 --warmup 1 > gpurun_out/alloc_bench.log 2>&1
rc=$?; echo "native-allocator bench rc=$rc"; grep -a '"metric"\|fault\|Memory access' gpurun_out/alloc_bench.log | cut -c1-400
if [ $rc -ne 0 ]; then python scripts/alloc_fault_map.py gpurun_out/alloc_trace.txt gpurun_out/alloc_bench.log; fi
ls -la gpurun_out/alloc_trace.txt
exit $rc
