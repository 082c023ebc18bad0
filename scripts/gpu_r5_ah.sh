#!/bin/bash
# Round 5 (ah): bias / norm-weight gradients into their fp32 main-grad slots — numerics vs fp32 sums, stage-3
# (short-circuit and forced-comm) training, then GPT-3 13B bf16 / fp8 and the Llama-2-7B headline with
# PADDLE2_AMD_BIAS_MAIN=1 / 0 on one box.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5ah
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_main_grad_1d_gpu.py tests/test_fp8_gpu.py tests/test_stage3_force_comm.py tests/test_bench_configs.py \
  $(ls tests/test_*norm*gpu*.py tests/test_*shard*gpu*.py 2>/dev/null) > $O/tests.log 2>&1
r=$?; tail -2 $O/tests.log; [ $r -ne 0 ] && { grep -E "^E |FAIL" $O/tests.log | head -30; exit $r; }
for d in 1 0; do
  PADDLE2_AMD_BIAS_MAIN=$d timeout -k 10 300 python -u bench.py --model gpt3-13b --seq-len 2048 --micro-batch 2 --steps 6 --warmup 3 > $O/bf16_13b_bm$d.log 2>&1
  r=$?; echo "13b bf16 bias_main=$d: $(tail -1 $O/bf16_13b_bm$d.log | cut -c1-150)"; [ $r -ne 0 ] && { tail -30 $O/bf16_13b_bm$d.log; exit $r; }
  tail -1 $O/bf16_13b_bm$d.log >> $O/bias_main.jsonl
  PADDLE2_AMD_BIAS_MAIN=$d timeout -k 10 300 python -u bench.py --model gpt3-13b --fp8 --seq-len 2048 --micro-batch 2 --steps 8 --warmup 3 > $O/fp8_13b_bm$d.log 2>&1
  r=$?; echo "13b fp8 bias_main=$d: $(tail -1 $O/fp8_13b_bm$d.log | cut -c1-150)"; [ $r -ne 0 ] && { tail -30 $O/fp8_13b_bm$d.log; exit $r; }
  tail -1 $O/fp8_13b_bm$d.log >> $O/bias_main.jsonl
done
timeout -k 10 400 python -u bench.py --steps 6 --warmup 3 > $O/llama.log 2>&1
r=$?; echo "llama: $(tail -1 $O/llama.log | cut -c1-150)"; [ $r -ne 0 ] && { tail -30 $O/llama.log; exit $r; }
tail -1 $O/llama.log >> $O/bias_main.jsonl
exit 0
