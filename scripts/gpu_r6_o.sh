#!/bin/bash
# Round 6 (o): secondary configs at HEAD — GPT-3 13B bf16, Llama-2-7B decode b1 / b16 / b64 serving.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6o
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
( while sleep 50; do date +%T >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 600 python -u bench.py --model gpt3-13b --seq-len 2048 --micro-batch 2 --steps 6 --warmup 2 > $O/gpt13b_bf16.log 2>&1
r=$?; tail -1 $O/gpt13b_bf16.log | cut -c1-220; [ $r -ne 0 ] && { kill $HB; tail -20 $O/gpt13b_bf16.log; exit $r; }
for b in 1 16 64; do
  timeout -k 10 400 python -u scripts/bench_serving.py --batch $b > $O/serve_b$b.json 2> $O/serve_b$b.err
  r=$?; tail -1 $O/serve_b$b.json; [ $r -ne 0 ] && { kill $HB; tail -20 $O/serve_b$b.err; exit $r; }
done
kill $HB
exit 0
