#!/bin/bash
# round-3 validation: full GPU test suite (native allocator now the default), smoke, bench, native RCCL PG worker
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/ \
    > gpurun_out/gpu_tests_r3.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_tests_r3.log; grep -c PASSED gpurun_out/gpu_tests_r3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/smoke_r3.log 2>&1
rc=$?; tail -2 gpurun_out/smoke_r3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench_r3.log 2>&1
rc=$?; grep '"metric"' gpurun_out/bench_r3.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
MASTER_PORT=29611 PD_TEST_OUT=gpurun_out/native_pg.json PYTHONPATH=. timeout -k 10 200 python -u -X faulthandler \
    tests/workers/native_pg_worker.py > gpurun_out/native_pg_worker.log 2>&1
rc=$?; echo "native pg worker rc=$rc"; tail -3 gpurun_out/native_pg_worker.log
exit $rc
