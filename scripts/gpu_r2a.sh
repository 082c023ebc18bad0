#!/bin/bash
# Round 2: headline bench on the stage-3 path (default) vs no wrapper, then the GPU suite.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r2a_bench_s3.log 2>&1
rc=$?; echo "bench s3 rc=$rc"; tail -2 gpurun_out/r2a_bench_s3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --sharding-stage 0 > gpurun_out/r2a_bench_s0.log 2>&1
rc=$?; echo "bench s0 rc=$rc"; tail -2 gpurun_out/r2a_bench_s0.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2a_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r2a_pytest_gpu.log
exit $rc
