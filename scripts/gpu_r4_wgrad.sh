#!/bin/bash
# Round 4: the spread schedule on the wgrad kernel (v5): GEMM GPU tests + bench.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4wg
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 900 python3 -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 300 --timeout-method thread > $O/gemm_tests.log 2>&1
rc=$?; echo "gemm tests rc=$rc"; tail -3 $O/gemm_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 -u scripts/bench_gemm_wgrad.py > $O/bench.jsonl 2> $O/bench.err
echo "bench rc=$?"; cat $O/bench.jsonl
