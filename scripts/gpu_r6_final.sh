#!/bin/bash
# Round 6 close-out at HEAD: the full GPU tier, smoke, the headline bench (the driver's default invocation), the GPT-3
# 13B bf16 / fp8 steps, decode b1 / b16 / b64, and a kernel table of the Llama-2-7B step.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6final
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
( while sleep 50; do date +%T >> $O/heartbeat.txt; done ) &
HB=$!
fail() { kill $HB; exit $1; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu tests \
  > $O/tests.log 2>&1
r=$?; tail -3 $O/tests.log; [ $r -ne 0 ] && { grep -E "^E |FAIL" $O/tests.log | head -30; fail $r; }
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1
r=$?; tail -2 $O/smoke.log; [ $r -ne 0 ] && { tail -30 $O/smoke.log; fail $r; }
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
r=$?; tail -1 $O/bench.log | cut -c1-300; [ $r -ne 0 ] && { tail -30 $O/bench.log; fail $r; }
timeout -k 10 600 python -u bench.py --model gpt3-13b --seq-len 2048 --micro-batch 2 --steps 8 --warmup 2 > $O/gpt13b_bf16.log 2>&1
r=$?; tail -1 $O/gpt13b_bf16.log | cut -c1-200; [ $r -ne 0 ] && { tail -30 $O/gpt13b_bf16.log; fail $r; }
timeout -k 10 600 python -u bench.py --model gpt3-13b --fp8 --seq-len 2048 --micro-batch 2 --steps 8 --warmup 2 > $O/gpt13b_fp8.log 2>&1
r=$?; tail -1 $O/gpt13b_fp8.log | cut -c1-200; [ $r -ne 0 ] && { tail -30 $O/gpt13b_fp8.log; fail $r; }
for b in 1 16 64; do
  timeout -k 10 400 python -u scripts/bench_serving.py --batch $b > $O/serve_b$b.json 2> $O/serve_b$b.err
  r=$?; echo "b$b $(grep -o '"decode_ms_per_step": [0-9.]*' $O/serve_b$b.json)"; [ $r -ne 0 ] && { tail -20 $O/serve_b$b.err; fail $r; }
done
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $O/prof_7b -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > $O/prof_7b.log 2>&1
r=$?; echo "prof 7b rc=$r"; [ $r -ne 0 ] && { tail -20 $O/prof_7b.log; fail $r; }
python3 scripts/kernel_table.py $(find $O/prof_7b -name "*kernel_trace.csv" | head -1) > $O/kernels_7b.txt 2>&1; head -22 $O/kernels_7b.txt
rm -f $(find $O/prof_7b -name "*kernel_trace.csv") 2>/dev/null
kill $HB
exit 0
