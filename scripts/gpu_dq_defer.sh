#!/bin/bash
# deferred dQ atomics: flash bwd ablation timing, flash GPU tests (all modes), headline bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/dqd
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_flash_dq_modes_gpu.py \
    tests/test_flash_gpu.py tests/test_flash_ext_gpu.py tests/test_llama_gpu.py > gpurun_out/dqd/tests.log 2>&1
rc=$?; tail -3 gpurun_out/dqd/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_flash_bwd_ablate.py > gpurun_out/dqd/ablate.jsonl 2> gpurun_out/dqd/err.log
rc=$?; cat gpurun_out/dqd/ablate.jsonl; tail -3 gpurun_out/dqd/err.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/dqd/bench.log 2>&1
rc=$?; grep '"metric"' gpurun_out/dqd/bench.log | cut -c1-300; exit $rc
