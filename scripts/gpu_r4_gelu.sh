#!/bin/bash
# Round 4: paddle.nn.functional.gelu on the native bias-activation kernel — tests and the GPT-3 13B bf16 step.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4gelu
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python3 -u -m pytest tests/test_fused_act.py -q -x -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $O/tests.log; [ $rc -ne 0 ] && [ $rc -ne 5 ] && exit $rc
timeout -k 10 600 python3 -u bench.py --model gpt3-13b --seq-len 2048 --micro-batch 2 --steps 5 --warmup 2 > $O/gpt13b_bf16.log 2>&1
r=$?; echo "gpt13b bf16 rc=$r"; grep -h '"metric"' $O/gpt13b_bf16.log | cut -c1-200; [ $r -ne 0 ] && { tail -20 $O/gpt13b_bf16.log; exit $r; }
exit 0
