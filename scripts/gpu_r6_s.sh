#!/bin/bash
# Round 6 (s): persistent MN-major wgrad (v7 SCHED bit 15) — GPU tests, isolated A/B vs v5, and the Llama / GPT-3 13B
# steps with it, plus the small-M forward route's tests.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
( while sleep 50; do date +%T >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_gemm_gpu.py \
  -k "wgrad_v7_mn or fwd_nn or schedule_variants or wgrad_fp32 or tail_splitk or identity" > $O/tests.log 2>&1
r=$?; tail -3 $O/tests.log; [ $r -ne 0 ] && { kill $HB; grep -E "^E |FAIL|Error" $O/tests.log | head -30; exit $r; }
timeout -k 10 400 python -u scripts/bench_wgrad_v7mn.py > $O/wgrad_ab.jsonl 2> $O/wgrad_ab.err
r=$?; cat $O/wgrad_ab.jsonl | cut -c1-200; [ $r -ne 0 ] && { kill $HB; tail -20 $O/wgrad_ab.err; exit $r; }
run() {  # name, env, args
  local n=$1; shift; local e=$1; shift
  env $e timeout -k 10 600 python -u bench.py "$@" > $O/$n.log 2>&1
  local r=$?; echo "$n $(tail -1 $O/$n.log | cut -c1-200)"; [ $r -ne 0 ] && { kill $HB; tail -20 $O/$n.log; exit $r; }
}
G="--model gpt3-13b --seq-len 2048 --micro-batch 2 --steps 8 --warmup 2"
run llama_mn PADDLE2_AMD_GEMM_VARIANT_WGRAD=33216 --steps 10 --warmup 3
run llama_v5 X=0 --steps 10 --warmup 3
run gpt_mn PADDLE2_AMD_GEMM_VARIANT_WGRAD=33216 $G
run gpt_v5 X=0 $G
kill $HB
exit 0
