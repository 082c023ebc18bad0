#!/bin/bash
# 8-wave flash forward: flash GPU tests, 4- vs 8-wave forward timing + bitwise check, bench.py
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 200 python -u scripts/bench_flash_fwd.py > gpurun_out/fa8_fwd.jsonl 2> gpurun_out/fa8_fwd.err
rc=$?; cat gpurun_out/fa8_fwd.jsonl; tail -3 gpurun_out/fa8_fwd.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_flash_gpu.py \
    tests/test_flash_ext_gpu.py tests/test_flash_dq_modes_gpu.py tests/test_llama_gpu.py > gpurun_out/fa8_tests.log 2>&1
rc=$?; tail -3 gpurun_out/fa8_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench_fa8.log 2>&1
rc=$?; grep '"metric"' gpurun_out/bench_fa8.log | cut -c1-400; exit $rc
