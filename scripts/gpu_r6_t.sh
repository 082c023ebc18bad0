#!/bin/bash
# Round 6 (t): persistent MN-major GEMMs (v7 SCHED bits 15 / 16) with precomputed transposed-read bases — GPU tests,
# isolated wgrad A/B vs v5, and the Llama / GPT-3 13B steps with the wgrad and the N-major forward on them.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6t
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
( while sleep 50; do date +%T >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_gemm_gpu.py \
  -k "wgrad_v7_mn or fwd_nn or schedule_variants or wgrad_fp32 or tail_splitk or identity or test_fwd" > $O/tests.log 2>&1
r=$?; tail -3 $O/tests.log; [ $r -ne 0 ] && { kill $HB; grep -E "^E |FAIL|Error" $O/tests.log | head -30; exit $r; }
timeout -k 10 400 python -u scripts/bench_wgrad_v7mn.py > $O/wgrad_ab.jsonl 2> $O/wgrad_ab.err
r=$?; grep '"beta": 0.0' $O/wgrad_ab.jsonl | cut -c1-150; [ $r -ne 0 ] && { kill $HB; tail -20 $O/wgrad_ab.err; exit $r; }
run() {  # name, env, args
  local n=$1; shift; local e=$1; shift
  env $e timeout -k 10 600 python -u bench.py "$@" > $O/$n.log 2>&1
  local r=$?; echo "$n $(tail -1 $O/$n.log | cut -c1-160)"; [ $r -ne 0 ] && { kill $HB; tail -20 $O/$n.log; exit $r; }
}
G="--model gpt3-13b --seq-len 2048 --micro-batch 2 --steps 8 --warmup 2"
MN=PADDLE2_AMD_GEMM_VARIANT_WGRAD=98752
NNF=PADDLE2_AMD_GEMM_VARIANT_FWD_NN=65984
run llama_base X=0 --steps 10 --warmup 3
run llama_mn $MN --steps 10 --warmup 3
run llama_mn_nnf "$MN $NNF PADDLE2_AMD_GEMM_FWD_NN_MAX_M=65536" --steps 10 --warmup 3
run gpt_base X=0 $G
run gpt_mn $MN $G
run gpt_mn_nnf "$MN $NNF" $G
run gpt_base2 X=0 $G
kill $HB
exit 0
