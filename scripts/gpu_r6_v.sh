#!/bin/bash
# Round 6 (v): flash backward wave-role options (PADDLE2_AMD_FA_BWD_OPT) at the Llama-2-7B shape.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6v
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python -u scripts/exp_flash_bwd_opt.py > $O/bwd_opt.jsonl 2> $O/bwd_opt.err
r=$?; cat $O/bwd_opt.jsonl; [ $r -ne 0 ] && { tail -20 $O/bwd_opt.err; exit $r; }
exit 0
