#!/bin/bash
# decode GEMM layout: serving GPU tests, layout microbench, end-to-end serving bench with the "nk" and "kn" layouts
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/nk
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_serving.py \
    > gpurun_out/nk/tests.log 2>&1
rc=$?; tail -2 gpurun_out/nk/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_skinny_gemm.py > gpurun_out/nk/gemm.jsonl 2> gpurun_out/nk/err.log
rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/bench_serving.py > gpurun_out/nk/serving_nk.log 2>&1
rc=$?; tail -1 gpurun_out/nk/serving_nk.log; [ $rc -eq 0 ] || exit $rc
PADDLE2_AMD_SERVING_LAYOUT=kn timeout -k 10 400 python -u scripts/bench_serving.py > gpurun_out/nk/serving_kn.log 2>&1
rc=$?; tail -1 gpurun_out/nk/serving_kn.log; exit $rc
