#!/bin/bash
# Round-2 measurements of the secondary configs on one MI355X: GPT-3 13B bf16 / fp8 (SURVEY config 5 slice),
# Llama-2-7B serving (paged KV, flash-decoding, HIP-graph decode), ResNet50 bf16 NHWC (config 2 slice).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/secondary
mkdir -p $O
for mode in "" "--fp8"; do
  tag=$([ -z "$mode" ] && echo bf16 || echo fp8)
  timeout -k 10 600 python bench.py --model gpt3-13b $mode --seq-len 2048 --micro-batch 2 --steps 5 --warmup 2 \
      > $O/gpt13b_$tag.log 2>&1
  rc=$?; echo "gpt13b $tag rc=$rc"; grep '"metric"' $O/gpt13b_$tag.log
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python scripts/bench_serving.py > $O/serving.log 2>&1
rc=$?; echo "serving rc=$rc"; tail -3 $O/serving.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/bench_resnet50.py --steps 20 --warmup 5 --batch 256 > $O/resnet50.json 2> $O/resnet50.err
rc=$?; echo "resnet rc=$rc"; cat $O/resnet50.json
exit $rc
