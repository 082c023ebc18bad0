#!/bin/bash
# Round 6 (ad): SwiGLU kernels with 4 rows per iteration vs 2 — isolated at the Llama shape, GPU tests under both, and
# the Llama step A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6ad
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python -u scripts/exp_swiglu_rows.py > $O/swiglu_rows.jsonl 2> $O/swiglu_rows.err
r=$?; cat $O/swiglu_rows.jsonl; [ $r -ne 0 ] && { tail -10 $O/swiglu_rows.err; exit $r; }
PADDLE2_AMD_SWIGLU_ROWS=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_kernels_gpu.py -k "swiglu" > $O/tests.log 2>&1
r=$?; tail -1 $O/tests.log; [ $r -ne 0 ] && { grep -E "^E |FAIL|Error" $O/tests.log | head -20; exit $r; }
run() {  # name, env, args
  local n=$1; shift; local e=$1; shift
  env $e timeout -k 10 600 python -u bench.py "$@" > $O/$n.log 2>&1
  local r=$?; echo "$n $(grep -o '"value": [0-9.]*' $O/$n.log | tail -1)"; [ $r -ne 0 ] && { tail -20 $O/$n.log; exit $r; }
}
run r4_a PADDLE2_AMD_SWIGLU_ROWS=4 --steps 10 --warmup 3
run r2_a X=0 --steps 10 --warmup 3
run r4_b PADDLE2_AMD_SWIGLU_ROWS=4 --steps 10 --warmup 3
run r2_b X=0 --steps 10 --warmup 3
exit 0
