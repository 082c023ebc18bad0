#!/bin/bash
# Native GEMM: numerics tests, then timing vs hipBLASLt on the Llama-2-7B shapes.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gemm_test.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/gemm_test.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_gemm_native.py > gpurun_out/gemm_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; cat gpurun_out/gemm_bench.log
exit $rc
