#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r3f
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest -x -q --timeout 450 --timeout-method thread -m gpu tests/test_dist_gpu.py \
    tests/test_flash_gpu.py tests/test_flash_ext_gpu.py > gpurun_out/r3f/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3f/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --model gpt3-13b --seq-len 2048 --micro-batch 2 --steps 3 --warmup 1 \
    > gpurun_out/r3f/gpt.log 2>&1
rc=$?; grep '"metric"' gpurun_out/r3f/gpt.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/r3f/bench.log 2>&1
rc=$?; grep '"metric"' gpurun_out/r3f/bench.log | cut -c1-300; exit $rc
