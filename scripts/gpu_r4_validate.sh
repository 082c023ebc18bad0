#!/bin/bash
# Round 4 validation of the new native paths: fp8 GEMM, GELU epilogues, 1x1 / 3x3 implicit-GEMM convs, v5 wgrad.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4val
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python3 -u -m pytest tests/test_fp8_gemm_gpu.py tests/test_fp8_gpu.py -x -q --timeout 120 --timeout-method thread > $O/fp8_tests.log 2>&1
rc=$?; echo "fp8 tests rc=$rc"; tail -4 $O/fp8_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u -m pytest tests/test_conv1x1_gpu.py tests/test_conv3x3_gpu.py -x -q --timeout 120 --timeout-method thread > $O/conv_tests.log 2>&1
rc=$?; echo "conv tests rc=$rc"; tail -4 $O/conv_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u -m pytest tests/test_rope_fold_gpu.py tests/test_flash_gpu.py -x -q --timeout 120 --timeout-method thread > $O/flash_tests.log 2>&1
rc=$?; echo "flash tests rc=$rc"; tail -4 $O/flash_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u -m pytest tests/test_decode_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/dec_tests.log 2>&1
rc=$?; echo "decode gemm tests rc=$rc"; tail -4 $O/dec_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 300 --timeout-method thread > $O/gemm_tests.log 2>&1
rc=$?; echo "gemm tests rc=$rc"; tail -4 $O/gemm_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u scripts/bench_gemm_fp8.py > $O/fp8_bench.jsonl 2> $O/fp8_bench.err
echo "fp8 bench rc=$?"; cat $O/fp8_bench.jsonl
timeout -k 10 300 python3 -u scripts/bench_gemm_wgrad.py > $O/wgrad_bench.jsonl 2> $O/wgrad_bench.err
echo "wgrad bench rc=$?"; cat $O/wgrad_bench.jsonl
timeout -k 10 300 python3 -u scripts/bench_decode_gemm.py > $O/dec_bench.jsonl 2> $O/dec_bench.err
echo "decode bench rc=$?"; cat $O/dec_bench.jsonl
exit 0
