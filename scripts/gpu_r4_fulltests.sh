#!/bin/bash
# The driver's round-end GPU tier, rehearsed: every gpu-marked test (one process, per-test timeout) and smoke().
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4full
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --maxfail 8 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -15 $O/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 $O/smoke.log
exit $rc
