#!/bin/bash
# Round 5 (aj): fp8 tests incl. the HIP-graph capture of the scale updates.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5aj
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_fp8_gpu.py tests/test_main_grad_1d_gpu.py > $O/tests.log 2>&1
r=$?; tail -3 $O/tests.log; [ $r -ne 0 ] && { grep -E "^E |FAIL" $O/tests.log | head -40; exit $r; }
exit 0
