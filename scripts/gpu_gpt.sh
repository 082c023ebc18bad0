#!/bin/bash
# GPT-3 13B (SURVEY config 5 slice) on one MI355X: bf16 vs fp8 linears, seq 2048.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for mode in "" "--fp8"; do
  tag=$([ -z "$mode" ] && echo bf16 || echo fp8)
  timeout -k 10 900 python bench.py --model gpt3-13b $mode --seq-len 2048 --micro-batch 2 --steps 3 --warmup 2 \
      > gpurun_out/gpt13b_$tag.log 2>&1
  rc=$?; echo "gpt13b $tag rc=$rc"; tail -2 gpurun_out/gpt13b_$tag.log
  [ $rc -eq 0 ] || exit $rc
done
