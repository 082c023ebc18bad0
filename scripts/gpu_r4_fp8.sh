#!/bin/bash
# Round 4: the native fp8 GEMM (gemm8.hip): GPU tests + bench vs hipBLASLt fp8 and bf16.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4fp8
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python3 -u -m pytest tests/test_fp8_gemm_gpu.py tests/test_fp8_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "fp8 tests rc=$rc"; tail -15 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u scripts/bench_gemm_fp8.py > $O/bench.jsonl 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cat $O/bench.jsonl; tail -3 $O/bench.err
exit $rc
