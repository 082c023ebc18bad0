#!/bin/bash
# Round 5 (e): fp8 GEMM late-wait schedule (PADDLE2_AMD_FP8_SCHED=1): numerics tests under it, then timing of both
# schedules vs hipBLASLt at the GPT-3 13B shapes.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5e
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
PADDLE2_AMD_FP8_SCHED=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_fp8_gemm_gpu.py tests/test_fp8_gpu.py tests/test_decode_gemm_gpu.py > $O/tests_s1.log 2>&1
r=$?; tail -3 $O/tests_s1.log; [ $r -ne 0 ] && { grep -E "^E |FAIL" $O/tests_s1.log | head -30; exit $r; }
timeout -k 10 200 python -u scripts/exp_fp8_cast.py > $O/fp8_cast.jsonl 2> $O/fp8_cast.err
r=$?; cat $O/fp8_cast.jsonl; [ $r -ne 0 ] && { tail -20 $O/fp8_cast.err; exit $r; }
for sc in 0 1; do
  PADDLE2_AMD_FP8_SCHED=$sc timeout -k 10 300 python -u scripts/bench_gemm_fp8.py > $O/fp8_s$sc.jsonl 2> $O/fp8_s$sc.err
  r=$?; cat $O/fp8_s$sc.jsonl; [ $r -ne 0 ] && { tail -20 $O/fp8_s$sc.err; exit $r; }
done
exit 0
