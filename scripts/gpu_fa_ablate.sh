#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/abl
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u scripts/bench_flash_bwd_ablate.py > gpurun_out/abl/fa_bwd_ablate.jsonl 2> gpurun_out/abl/err.log
rc=$?; cat gpurun_out/abl/fa_bwd_ablate.jsonl; tail -3 gpurun_out/abl/err.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_flash_dq_modes_gpu.py \
    tests/test_flash_gpu.py > gpurun_out/abl/tests.log 2>&1
rc=$?; tail -2 gpurun_out/abl/tests.log; exit $rc
