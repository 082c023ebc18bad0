#!/bin/bash
# Round 6 (i): widened (16-B) forward O stores — flash GPU tests at HEAD, then the forward timing A/B against the
# previous build (abtest/, same box, interleaved), then the step with the default route.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6i
mkdir -p $O
export TMPDIR=/tmp
PYTHONPATH=$PWD timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_flash_fwd_rb2_gpu.py tests/test_flash_gpu.py tests/test_flash_ext_gpu.py tests/test_flash_dq_split_gpu.py tests/test_flash_dq_modes_gpu.py > $O/tests.log 2>&1
r=$?; tail -3 $O/tests.log; [ $r -ne 0 ] && { grep -E "^E |FAIL|Error" $O/tests.log | head -30; exit $r; }
for rnd in 0 1; do
  for v in old new; do
    if [ $v = old ]; then P=$PWD/abtest; else P=$PWD; fi
    PYTHONPATH=$P ROUNDS=1 timeout -k 10 300 python -u scripts/bench_flash_fwd_rb.py > $O/fwd_${v}_$rnd.jsonl 2> $O/fwd_$v.err
    r=$?; [ $r -ne 0 ] && { tail -20 $O/fwd_$v.err; exit $r; }
    sed "s/^{/{\"build\": \"$v\", /" $O/fwd_${v}_$rnd.jsonl
  done
done
exit 0
