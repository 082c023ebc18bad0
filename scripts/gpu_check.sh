#!/bin/bash
# Round-end style validation on one MI355X: GPU tests, smoke, default bench. Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
if [ "${SKIP_BENCH:-0}" = "0" ]; then
  timeout -k 10 900 python -u bench.py > gpurun_out/bench_default.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_default.log
  exit $rc
fi
