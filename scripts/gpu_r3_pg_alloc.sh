#!/bin/bash
# 7B bench on the native allocator (allocation trace on) after the GEMM tests, then the native RCCL PG test
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash scripts/gpu_alloc_r3.sh; arc=$?
echo "alloc rc=$arc"
[ $arc -eq 0 ] || exit $arc
MASTER_PORT=29611 PD_TEST_OUT=gpurun_out/native_pg.json PYTHONPATH=. timeout -k 10 200 python -u -X faulthandler tests/workers/native_pg_worker.py \
    > gpurun_out/native_pg_worker.log 2>&1
rc=$?; echo "native pg worker rc=$rc"; tail -40 gpurun_out/native_pg_worker.log
exit $rc
