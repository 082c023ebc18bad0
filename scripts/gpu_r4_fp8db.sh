#!/bin/bash
# Round 4: fp8 linear bias gradient on the native column sum — fp8 GPU tests and the GPT-3 13B fp8 step.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4fp8db
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python3 -u -m pytest tests/test_fp8_gpu.py tests/test_fp8_gemm_gpu.py -q -x -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 -u bench.py --model gpt3-13b --fp8 --seq-len 2048 --micro-batch 2 --steps 5 --warmup 2 > $O/gpt13b_fp8.log 2>&1
r=$?; echo "gpt13b fp8 rc=$r"; grep -h '"metric"' $O/gpt13b_fp8.log | cut -c1-200; exit $r
