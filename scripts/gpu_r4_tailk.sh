#!/bin/bash
# Round 4: the v7 tail split-K — numerics, GEMM timing at the GPT-3 13B / Llama shapes with and without it, and the
# GPT-3 13B + Llama-2-7B steps.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4tailk
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python3 -u -m pytest tests/test_gemm_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "tail_splitk or gelu_mlp or llama7b_shapes" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u scripts/bench_tailk.py > $O/gemm.jsonl 2> $O/gemm.err
rc=$?; echo "gemm rc=$rc"; cat $O/gemm.jsonl; [ $rc -ne 0 ] && { tail -20 $O/gemm.err; exit $rc; }
timeout -k 10 600 python3 -u bench.py --model gpt3-13b --seq-len 2048 --micro-batch 2 --steps 5 --warmup 2 > $O/gpt13b_bf16.log 2>&1
r=$?; echo "gpt13b bf16 rc=$r"; grep -h '"metric"' $O/gpt13b_bf16.log | cut -c1-200; [ $r -ne 0 ] && { tail -20 $O/gpt13b_bf16.log; exit $r; }
timeout -k 10 420 python3 -u bench.py --steps 10 --warmup 3 > $O/bench.log 2>&1
r=$?; echo "bench rc=$r"; grep -h '"metric"' $O/bench.log | cut -c1-250; [ $r -ne 0 ] && { tail -20 $O/bench.log; exit $r; }
exit 0
