#!/bin/bash
# Round 6 (d): split-dQ numerics + timing + kernel table after the barrier / load-issue fixes.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6d
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_flash_dq_split_gpu.py \
  > $O/tests.log 2>&1
r=$?; tail -3 $O/tests.log; [ $r -ne 0 ] && { grep -E "^E " $O/tests.log | head -30; exit $r; }
timeout -k 10 300 python -u scripts/bench_flash_bwd_ablate.py > $O/fa_bwd_ablate.jsonl 2> $O/abl_err.log
r=$?; cat $O/fa_bwd_ablate.jsonl; [ $r -ne 0 ] && { tail -10 $O/abl_err.log; exit $r; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/prof_flash_bwd_split.py 1 > $O/prof.log 2>&1
r=$?; [ $r -ne 0 ] && { tail -20 $O/prof.log; exit $r; }
rm -f $(find $O/prof -name "*kernel_trace.csv") 2>/dev/null
exit 0
