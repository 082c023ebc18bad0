#!/bin/bash
# native RCCL process group (1 rank) + GEMM tests + 7B bench on the native allocator (allocation trace on)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_native_pg_gpu.py \
    > gpurun_out/native_pg_tests.log 2>&1
rc=$?; tail -4 gpurun_out/native_pg_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_alloc_r3.sh
