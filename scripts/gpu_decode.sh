#!/bin/bash
# decode kernels: GPU tests (vector + MFMA) then the kernel benchmark
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_serving.py \
    > gpurun_out/decode_tests.log 2>&1
rc=$?; tail -5 gpurun_out/decode_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_decode.py > gpurun_out/decode_bench.jsonl 2>&1
rc=$?; cat gpurun_out/decode_bench.jsonl; exit $rc
