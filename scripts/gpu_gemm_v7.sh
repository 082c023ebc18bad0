#!/bin/bash
# v7 GEMM: GPU tests (gemm file only) then the shape benchmark vs v4/v6/hipBLASLt
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gemm_gpu.py \
    > gpurun_out/gemm_v7_tests.log 2>&1
rc=$?; tail -5 gpurun_out/gemm_v7_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_gemm_v7.py 7,8,9,10 > gpurun_out/gemm_v7_bench.jsonl 2> gpurun_out/gemm_v7_bench.err
rc=$?; cat gpurun_out/gemm_v7_bench.jsonl | cut -c1-200; tail -3 gpurun_out/gemm_v7_bench.err; exit $rc
