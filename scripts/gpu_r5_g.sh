#!/bin/bash
# Round 5 (g): MFMA shape study (16x16x32 vs 32x32x16, GEMM wave tile, random data), fp8 GEMM schedules 0 / 1 vs
# hipBLASLt at the GPT-3 13B shapes (sched 2 = spread LDS-DMA pieces, numerics-tested first), and one PMC pass per fp8 implementation at 8192^3.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5g
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 120 ./scripts/mfma_shape > $O/mfma_shape.jsonl 2> $O/mfma_shape.err
r=$?; cat $O/mfma_shape.jsonl; [ $r -ne 0 ] && { tail -20 $O/mfma_shape.err; exit $r; }
PADDLE2_AMD_FP8_SCHED=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_fp8_gemm_gpu.py tests/test_fp8_gpu.py tests/test_decode_gemm_gpu.py > $O/tests_s2.log 2>&1
r=$?; tail -2 $O/tests_s2.log; [ $r -ne 0 ] && { grep -E "^E |FAIL" $O/tests_s2.log | head -30; exit $r; }
for sc in 0 1 2; do
  PADDLE2_AMD_FP8_SCHED=$sc timeout -k 10 300 python -u scripts/bench_gemm_fp8.py > $O/fp8_s$sc.jsonl 2> $O/fp8_s$sc.err
  r=$?; cat $O/fp8_s$sc.jsonl; [ $r -ne 0 ] && { tail -20 $O/fp8_s$sc.err; exit $r; }
done
CTR="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
for impl in native blas; do
  timeout -s KILL 90 rocprofv3 --pmc $CTR -d $O/pmc_$impl -o run --output-format csv -- python3 scripts/prof_fp8.py $impl 8192 8192 8192 \
    > $O/pmc_$impl.log 2>&1
  r=$?; echo "pmc $impl rc=$r"; [ $r -ne 0 ] && { tail -20 $O/pmc_$impl.log; exit $r; }
done
timeout -s KILL 90 rocprofv3 --pmc $CTR -d $O/pmc_native1 -o run --output-format csv -- python3 scripts/prof_fp8.py native 8192 8192 8192 1 \
  > $O/pmc_native1.log 2>&1
r=$?; echo "pmc native sched1 rc=$r"; [ $r -ne 0 ] && { tail -20 $O/pmc_native1.log; exit $r; }
timeout -k 10 300 python -u scripts/exp_decode64.py > $O/dec64.jsonl 2> $O/dec64.err
r=$?; cat $O/dec64.jsonl; [ $r -ne 0 ] && { tail -20 $O/dec64.err; exit $r; }
timeout -k 10 300 python -u scripts/bench_serving.py --batch 64 > $O/serving_b64.log 2>&1
r=$?; tail -2 $O/serving_b64.log; [ $r -ne 0 ] && { tail -20 $O/serving_b64.log; exit $r; }
PADDLE2_AMD_DECODE_GEMM=blas timeout -k 10 300 python -u scripts/bench_serving.py --batch 64 > $O/serving_b64_blas.log 2>&1
r=$?; tail -2 $O/serving_b64_blas.log; [ $r -ne 0 ] && { tail -20 $O/serving_b64_blas.log; exit $r; }
exit 0
