#!/bin/bash
# Round 5 (y): fp8 GEMM tile-group height sweep with the bias epilogue vs hipBLASLt at the GPT-3 13B shapes.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5y
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python -u scripts/exp_fp8_groupm.py > $O/groupm.jsonl 2> $O/groupm.err
r=$?; cat $O/groupm.jsonl; [ $r -ne 0 ] && { tail -20 $O/groupm.err; exit $r; }
exit 0
