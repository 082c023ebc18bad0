#!/bin/bash
# Round 4: tail split-K on the bf16 (v7) and fp8 GEMMs — numerics, GEMM timings, GPT-3 13B bf16 / fp8 steps.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4tailk2
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python3 -u -m pytest tests/test_gemm_gpu.py tests/test_fp8_gemm_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u scripts/bench_tailk.py > $O/gemm.jsonl 2> $O/gemm.err
rc=$?; echo "gemm rc=$rc"; cat $O/gemm.jsonl; [ $rc -ne 0 ] && { tail -20 $O/gemm.err; exit $rc; }
for g in native auto; do
  PADDLE2_AMD_FP8_GEMM=$g timeout -k 10 600 python3 -u bench.py --model gpt3-13b --fp8 --seq-len 2048 --micro-batch 2 --steps 5 --warmup 2 > $O/gpt13b_fp8_$g.log 2>&1
  r=$?; echo "gpt13b fp8 $g rc=$r"; grep -h '"metric"' $O/gpt13b_fp8_$g.log | cut -c1-200; [ $r -ne 0 ] && { tail -20 $O/gpt13b_fp8_$g.log; exit $r; }
done
timeout -k 10 600 python3 -u bench.py --model gpt3-13b --seq-len 2048 --micro-batch 2 --steps 5 --warmup 2 --gemm-route static > $O/gpt13b_bf16_static.log 2>&1
r=$?; echo "gpt13b bf16 static rc=$r"; grep -h '"metric"' $O/gpt13b_bf16_static.log | cut -c1-200; [ $r -ne 0 ] && { tail -20 $O/gpt13b_bf16_static.log; exit $r; }
timeout -k 10 600 python3 -u bench.py --model gpt3-13b --seq-len 2048 --micro-batch 2 --steps 5 --warmup 2 > $O/gpt13b_bf16.log 2>&1
r=$?; echo "gpt13b bf16 rc=$r"; grep -h '"metric"' $O/gpt13b_bf16.log | cut -c1-200; exit $r
