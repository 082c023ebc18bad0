#!/bin/bash
# Round 5 (r): the LDS-X decode kernel (dec64s) — numerics vs fp32 at every configuration, then the bandwidth sweep
# against dec64 (register X) and hipBLASLt at M = 24 / 32 / 48 / 64 on the Llama-2-7B projections.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5r
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_decode_gemm_gpu.py > $O/tests.log 2>&1
r=$?; tail -2 $O/tests.log; [ $r -ne 0 ] && { grep -E "^E |FAIL" $O/tests.log | head -30; exit $r; }
timeout -k 10 400 python -u scripts/exp_decode64.py > $O/dec64.jsonl 2> $O/dec64.err
r=$?; cat $O/dec64.jsonl | cut -c1-600; [ $r -ne 0 ] && { tail -20 $O/dec64.err; exit $r; }
exit 0
