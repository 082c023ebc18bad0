#!/bin/bash
# Round 6 (w): tile-group height of the N-major forward and the MN-major weight gradient at the Llama shapes.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6w
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python -u scripts/exp_gemm_groupm_r6.py > $O/groupm.jsonl 2> $O/groupm.err
r=$?; cat $O/groupm.jsonl | cut -c1-120; [ $r -ne 0 ] && { tail -20 $O/groupm.err; exit $r; }
exit 0
