#!/bin/bash
# GEMM tests, then the headline bench (default per-pass GEMM routing) and the all-native variant.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2b_gemm_test.log 2>&1
rc=$?; echo "gemm tests rc=$rc"; tail -3 gpurun_out/r2b_gemm_test.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r2b_bench_default.log 2>&1
rc=$?; echo "bench default rc=$rc"; tail -1 gpurun_out/r2b_bench_default.log
[ $rc -eq 0 ] || exit $rc
PADDLE2_AMD_GEMM_FWD=native PADDLE2_AMD_GEMM_DGRAD=native timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r2b_bench_allnative.log 2>&1
rc=$?; echo "bench all-native rc=$rc"; tail -1 gpurun_out/r2b_bench_allnative.log
PADDLE2_AMD_GEMM_WGRAD=blas timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r2b_bench_allblas.log 2>&1
rc=$?; echo "bench all-blas rc=$rc"; tail -1 gpurun_out/r2b_bench_allblas.log
exit $rc
