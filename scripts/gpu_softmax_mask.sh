#!/bin/bash
# New fused masked-softmax kernel: GPU numerics tests, micro-benchmark, kernel trace.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_softmax_mask.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_sm.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_sm.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_softmax_mask.py > gpurun_out/bench_sm.log 2>&1
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_sm.log | tail -8
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_sm" -o sm -- python3 "$GRAFT_REPO_ROOT/scripts/bench_softmax_mask.py" > "$GRAFT_REPO_ROOT/gpurun_out/prof_sm.log" 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
