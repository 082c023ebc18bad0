#!/bin/bash
# Round 6 end: after the decode split-target change: the full GPU tier, smoke and the headline bench.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6end
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu tests \
  > $O/tests.log 2>&1
r=$?; tail -3 $O/tests.log; [ $r -ne 0 ] && { grep -E "^E |FAIL" $O/tests.log | head -30; exit $r; }
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1
r=$?; tail -2 $O/smoke.log; [ $r -ne 0 ] && { tail -30 $O/smoke.log; exit $r; }
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
r=$?; tail -1 $O/bench.log | cut -c1-300; [ $r -ne 0 ] && { tail -30 $O/bench.log; exit $r; }
exit 0
