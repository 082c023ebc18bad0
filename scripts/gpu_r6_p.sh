#!/bin/bash
# Round 6 (p): 16x16x32 flash forward + RB=2 — numerics, then RB = 1 vs RB = 2 timing.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6p
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_flash_fwd_rb2_gpu.py > $O/tests.log 2>&1
r=$?; tail -3 $O/tests.log; [ $r -ne 0 ] && { grep -E "^E |Error" $O/tests.log | head -30; exit $r; }
timeout -k 10 300 python -u scripts/bench_flash_fwd_rb.py > $O/fwd_rb.jsonl 2> $O/fwd_rb.err
r=$?; cat $O/fwd_rb.jsonl; [ $r -ne 0 ] && { tail -20 $O/fwd_rb.err; exit $r; }
exit 0
