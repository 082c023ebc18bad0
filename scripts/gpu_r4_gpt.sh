#!/bin/bash
# Round 4: GPT-3 13B (seq 2048, micro-batch 2, one GPU) with and without the fused GELU-MLP node.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4gpt
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
for f in 1 0; do
  PADDLE2_AMD_FUSED_GELU_MLP=$f timeout -k 10 600 python3 -u bench.py --model gpt3-13b --seq-len 2048 --micro-batch 2 --steps 5 --warmup 2 > $O/gpt13b_fused$f.log 2>&1
  rc=$?; echo "gpt13b fused=$f rc=$rc"; grep '"metric"' $O/gpt13b_fused$f.log | cut -c1-250; [ $rc -ne 0 ] && exit $rc
done
exit 0
