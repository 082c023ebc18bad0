#!/bin/bash
# session-3 check: GEMM GPU tests, v7 shape benchmark, bench.py (default routing)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gemm_gpu.py \
    > gpurun_out/gemm_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gemm_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_gemm_v7.py 7,8,9,10 > gpurun_out/gemm_v7_bench.jsonl 2> gpurun_out/gemm_v7_bench.err
rc=$?; cut -c1-160 gpurun_out/gemm_v7_bench.jsonl; tail -3 gpurun_out/gemm_v7_bench.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench_r3c.log 2>&1
rc=$?; grep '"metric"' gpurun_out/bench_r3c.log | cut -c1-600; exit $rc
