#!/bin/bash
# Round 6 (af): flash backward dispatch order at the Llama shape — heaviest key blocks first (default) vs a (b, kv head)
# pair's key blocks co-dispatched on one XCD (PADDLE2_AMD_FA_BWD_ORDER=pair).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6af
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python -u scripts/exp_flash_bwd_opt.py heavy,pair > $O/bwd_order.jsonl 2> $O/bwd_order.err
r=$?; cat $O/bwd_order.jsonl; [ $r -ne 0 ] && { tail -10 $O/bwd_order.err; exit $r; }
exit 0
