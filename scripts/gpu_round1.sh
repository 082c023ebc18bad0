#!/bin/bash
# First GPU validation: kernel numerics, smoke, small + full benches. Stops at the first fault.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
ok $rc || exit $rc
timeout -k 10 600 python bench.py --layers 4 --steps 3 --warmup 1 --micro-batch 1 > gpurun_out/bench_L4.log 2>&1
rc=$?; echo "bench L4 rc=$rc"; tail -5 gpurun_out/bench_L4.log
ok $rc || exit $rc
timeout -k 10 900 python bench.py --steps 3 --warmup 2 --micro-batch 1 > gpurun_out/bench_7b_b1.log 2>&1
rc=$?; echo "bench 7b b1 rc=$rc"; tail -5 gpurun_out/bench_7b_b1.log
