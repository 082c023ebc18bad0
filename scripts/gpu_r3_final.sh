#!/bin/bash
# round-3 final validation: full GPU suite, smoke, headline bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/final
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ \
    > gpurun_out/final/gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/final/gpu_tests.log; grep -c PASSED gpurun_out/final/gpu_tests.log; grep -E "FAILED|ERROR" gpurun_out/final/gpu_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/final/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/final/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/final/bench.log 2>&1
rc=$?; tail -1 gpurun_out/final/bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/bench_serving.py > gpurun_out/final/serving.log 2>&1
rc=$?; tail -1 gpurun_out/final/serving.log; exit $rc
