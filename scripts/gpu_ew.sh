#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ew
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 200 python -u scripts/bench_swiglu.py > gpurun_out/ew/swiglu.jsonl 2> gpurun_out/ew/err.log
rc=$?; cat gpurun_out/ew/swiglu.jsonl; tail -3 gpurun_out/ew/err.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/bench_rope.py > gpurun_out/ew/rope.jsonl 2>> gpurun_out/ew/err.log
rc=$?; cat gpurun_out/ew/rope.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
    tests/test_fused_act.py tests/test_llama_gpu.py tests/test_flash_gpu.py > gpurun_out/ew/tests.log 2>&1
rc=$?; tail -3 gpurun_out/ew/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/ew/bench.log 2>&1
rc=$?; grep '"metric"' gpurun_out/ew/bench.log | cut -c1-300; exit $rc
