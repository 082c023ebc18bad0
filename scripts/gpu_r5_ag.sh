#!/bin/bash
# Round 5 (ag): deferred fp8 scale updates (16 roles per launch) — fp8 numerics incl. the deferred-vs-immediate
# parity test, the GPT-3 13B fp8 step with PADDLE2_AMD_FP8_DEFER=1 / 0 on one box, and the default's kernel table.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5ag
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_fp8_gpu.py tests/test_fp8_gemm_gpu.py tests/test_bench_configs.py > $O/tests.log 2>&1
r=$?; tail -2 $O/tests.log; [ $r -ne 0 ] && { grep -E "^E |FAIL" $O/tests.log | head -30; exit $r; }
for d in 1 0 1; do
  PADDLE2_AMD_FP8_DEFER=$d timeout -k 10 300 python -u bench.py --model gpt3-13b --fp8 --seq-len 2048 --micro-batch 2 --steps 8 --warmup 3 > $O/fp8_13b_defer$d.log 2>&1
  r=$?; echo "defer=$d: $(tail -1 $O/fp8_13b_defer$d.log | cut -c1-160)"; [ $r -ne 0 ] && { tail -30 $O/fp8_13b_defer$d.log; exit $r; }
  tail -1 $O/fp8_13b_defer$d.log >> $O/fp8_13b_defer.jsonl
done
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $O/prof_fp8 -o run --output-format csv -- python3 bench.py --model gpt3-13b --fp8 --seq-len 2048 --micro-batch 2 --steps 3 --warmup 2 > $O/prof_fp8.log 2>&1
r=$?; echo "prof rc=$r"; [ $r -ne 0 ] && { tail -20 $O/prof_fp8.log; exit $r; }
python3 scripts/kernel_table.py $(find $O/prof_fp8 -name "*kernel_trace.csv" | head -1) > $O/kernels_fp8.txt 2>&1; head -30 $O/kernels_fp8.txt
rm -f $(find $O/prof_fp8 -name "*kernel_trace.csv") 2>/dev/null
exit 0
