#!/bin/bash
# Full GPU suite + smoke after the masked-softmax / MoE changes, then a kernel-trace profile of the
# masked-softmax micro-benchmark. Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_sm" -o sm -- python3 "$GRAFT_REPO_ROOT/scripts/bench_softmax_mask.py" > "$GRAFT_REPO_ROOT/gpurun_out/prof_sm.log" 2>&1
rc=$?; echo "prof rc=$rc"; tail -3 "$GRAFT_REPO_ROOT/gpurun_out/prof_sm.log"; exit $rc
