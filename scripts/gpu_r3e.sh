#!/bin/bash
# fwd wave-skip experiment, packed-QKV + 2-rank single-GPU tests, GPT-3 13B bench after the packed-QKV path
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r3e
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u scripts/bench_flash_fwd.py > gpurun_out/r3e/fwd.jsonl 2> gpurun_out/r3e/fwd.err
rc=$?; cat gpurun_out/r3e/fwd.jsonl; tail -3 gpurun_out/r3e/fwd.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 450 --timeout-method thread -m gpu tests/test_flash_gpu.py \
    tests/test_dist_gpu.py > gpurun_out/r3e/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3e/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --model gpt3-13b --seq-len 2048 --micro-batch 2 --steps 3 --warmup 1 \
    > gpurun_out/r3e/gpt.log 2>&1
rc=$?; grep '"metric"' gpurun_out/r3e/gpt.log | cut -c1-300; exit $rc
