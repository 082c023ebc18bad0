#!/bin/bash
# Round 6 (a): baseline on this round's first box — the headline bench and the flash backward dQ-path ablation.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6a
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
r=$?; tail -1 $O/bench.log | cut -c1-400; [ $r -ne 0 ] && { tail -30 $O/bench.log; exit $r; }
timeout -k 10 300 python -u scripts/bench_flash_bwd_ablate.py > $O/fa_bwd_ablate.jsonl 2> $O/abl_err.log
r=$?; cat $O/fa_bwd_ablate.jsonl; [ $r -ne 0 ] && { tail -10 $O/abl_err.log; exit $r; }
exit 0
