#!/bin/bash
# Round 5 (ac): SwiGLU folded into the decode down GEMM (<= 16 rows) — serving / decode GPU tests, then the decode
# step at b1 / b16 / b64.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5ac
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_serving.py tests/test_decode_gemm_gpu.py > $O/tests.log 2>&1
r=$?; tail -2 $O/tests.log; [ $r -ne 0 ] && { grep -E "^E |FAIL" $O/tests.log | head -30; exit $r; }
for b in 1 16 64; do
  timeout -k 10 300 python -u scripts/bench_serving.py --batch $b > $O/serving_b$b.log 2>&1
  r=$?; echo "b$b: $(grep '^{' $O/serving_b$b.log | cut -c1-260)"; [ $r -ne 0 ] && { tail -20 $O/serving_b$b.log; exit $r; }
done
exit 0
