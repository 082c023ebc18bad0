#!/bin/bash
# Round 5 (q): full GPU tier at HEAD (allocator OOM fix, fp8 schedule 2 + fp32 wgrad-into-main defaults, one-wave fp8
# scale update, dec64 channel tiles, serving decode through the native decode GEMM), smoke, the dec64 channel-tile
# sweep vs hipBLASLt, the serving decode step at b1 / b16 / b64 (default routing vs hipBLASLt) and the GPT-3 13B fp8
# step on the new defaults.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5q
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu tests \
  > $O/tests.log 2>&1
r=$?; tail -3 $O/tests.log; [ $r -ne 0 ] && { grep -E "^E |FAIL" $O/tests.log | head -30; exit $r; }
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1
r=$?; tail -2 $O/smoke.log; [ $r -ne 0 ] && { tail -30 $O/smoke.log; exit $r; }
timeout -k 10 300 python -u scripts/exp_decode64.py > $O/dec64.jsonl 2> $O/dec64.err
r=$?; cat $O/dec64.jsonl | cut -c1-330; [ $r -ne 0 ] && { tail -20 $O/dec64.err; exit $r; }
for b in 1 16 64; do
  timeout -k 10 300 python -u scripts/bench_serving.py --batch $b > $O/serving_b$b.log 2>&1
  r=$?; echo "b$b native: $(grep '^{' $O/serving_b$b.log | cut -c1-250)"; [ $r -ne 0 ] && { tail -20 $O/serving_b$b.log; exit $r; }
  PADDLE2_AMD_DECODE_GEMM=blas timeout -k 10 300 python -u scripts/bench_serving.py --batch $b > $O/serving_b${b}_blas.log 2>&1
  r=$?; echo "b$b blas: $(grep '^{' $O/serving_b${b}_blas.log | cut -c1-250)"; [ $r -ne 0 ] && { tail -20 $O/serving_b${b}_blas.log; exit $r; }
done
timeout -k 10 300 python -u bench.py --model gpt3-13b --fp8 --seq-len 2048 --micro-batch 2 --steps 8 --warmup 3 > $O/fp8_13b.log 2>&1
r=$?; echo "fp8 13b: $(tail -1 $O/fp8_13b.log | cut -c1-200)"; [ $r -ne 0 ] && { tail -30 $O/fp8_13b.log; exit $r; }
exit 0
