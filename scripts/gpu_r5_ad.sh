#!/bin/bash
# Round 5 (ad): packed (batched varlen) prefill — serving GPU tests, then prefill + decode at b64 / b16 with the
# packed prefill vs one prompt at a time.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5ad
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_serving.py > $O/tests.log 2>&1
r=$?; tail -2 $O/tests.log; [ $r -ne 0 ] && { grep -E "^E |FAIL" $O/tests.log | head -30; exit $r; }
for v in "b64_batch:--batch 64 --prefill batch" "b64_seq:--batch 64 --prefill seq" "b16_batch:--batch 16 --prefill batch"; do
  name=${v%%:*}; a=${v#*:}
  timeout -k 10 300 python -u scripts/bench_serving.py $a > $O/$name.log 2>&1
  r=$?; echo "$name: $(grep '^{' $O/$name.log | cut -c1-300)"; [ $r -ne 0 ] && { tail -20 $O/$name.log; exit $r; }
done
exit 0
