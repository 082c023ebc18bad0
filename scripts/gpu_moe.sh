#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_fused_moe.py \
  tests/test_incubate_attention.py tests/test_gemm_gpu.py tests/test_serving.py > gpurun_out/moe_tests.log 2>&1
rc=$?; tail -4 gpurun_out/moe_tests.log; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_moe.py > gpurun_out/moe_bench.log 2>&1
rc=$?; cat gpurun_out/moe_bench.log | tail -5; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_gemm_native.py 32768 0 > gpurun_out/gemm_bench_r2c.log 2>&1
rc=$?; cat gpurun_out/gemm_bench_r2c.log; echo "gemm rc=$rc"; exit $rc
