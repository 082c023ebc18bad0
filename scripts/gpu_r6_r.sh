#!/bin/bash
# Round 6 (r): forward GEMM on W as stored with the spread schedule (variant 5, B operand N-major through transposed
# LDS reads, no per-step W^T) vs the TN default (v7 on W^T): GPT-3 13B bf16 (M = 4096 tokens) and Llama-2-7B (32768).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6r
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
( while sleep 50; do date +%T >> $O/heartbeat.txt; done ) &
HB=$!
run() {  # name, env, args
  local n=$1; shift; local e=$1; shift
  env $e timeout -k 10 600 python -u bench.py "$@" > $O/$n.log 2>&1
  local r=$?; echo "$n $(tail -1 $O/$n.log | cut -c1-200)"; [ $r -ne 0 ] && { kill $HB; tail -20 $O/$n.log; exit $r; }
}
G="--model gpt3-13b --seq-len 2048 --micro-batch 2 --steps 8 --warmup 2"
run gpt_v7a X=0 $G
run gpt_v5a PADDLE2_AMD_GEMM_VARIANT_FWD=5 $G
run gpt_v7b X=0 $G
run gpt_v5b PADDLE2_AMD_GEMM_VARIANT_FWD=5 $G
run llama_v5 PADDLE2_AMD_GEMM_VARIANT_FWD=5 --steps 10 --warmup 3
run llama_v7 X=0 --steps 10 --warmup 3
kill $HB
exit 0
