#!/bin/bash
# Round 6 (b): split-dQ flash backward — numerics against fp32, then the dQ-path timing at the Llama-2-7B shape.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6b
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_flash_dq_split_gpu.py \
  > $O/tests.log 2>&1
r=$?; tail -12 $O/tests.log; [ $r -ne 0 ] && { grep -E "^E " $O/tests.log | head -30; exit $r; }
timeout -k 10 300 python -u scripts/bench_flash_bwd_ablate.py > $O/fa_bwd_ablate.jsonl 2> $O/abl_err.log
r=$?; cat $O/fa_bwd_ablate.jsonl; [ $r -ne 0 ] && { tail -10 $O/abl_err.log; exit $r; }
exit 0
