#!/bin/bash
# Round 5 (f): re-validate HEAD after the session restart — the full GPU tier, smoke, the 7B bench (default and
# forced-comm stage 3), and a kernel table of the default step.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5f
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu tests \
  > $O/tests.log 2>&1
r=$?; tail -3 $O/tests.log; [ $r -ne 0 ] && { grep -E "^E |FAIL" $O/tests.log | head -30; exit $r; }
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1
r=$?; tail -2 $O/smoke.log; [ $r -ne 0 ] && { tail -30 $O/smoke.log; exit $r; }
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > $O/bench_plain.log 2>&1
r=$?; tail -1 $O/bench_plain.log; [ $r -ne 0 ] && { tail -30 $O/bench_plain.log; exit $r; }
PADDLE2_AMD_STAGE3_FORCE_COMM=1 timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > $O/bench_force.log 2>&1
r=$?; tail -1 $O/bench_force.log; [ $r -ne 0 ] && { tail -30 $O/bench_force.log; exit $r; }
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > $O/prof.log 2>&1
r=$?; echo "prof rc=$r"; [ $r -ne 0 ] && { tail -20 $O/prof.log; exit $r; }
python3 scripts/kernel_table.py $(find $O/prof -name "*kernel_trace.csv" | head -1) > $O/kernels.txt 2>&1; head -40 $O/kernels.txt
rm -f $(find $O/prof -name "*kernel_trace.csv") 2>/dev/null
exit 0
