#!/bin/bash
# Round 6 (f): close-out at HEAD — the full GPU tier, smoke, the headline bench (N = 1, the driver's default
# invocation), and a kernel table of the Llama-2-7B step.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6f
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu tests \
  > $O/tests.log 2>&1
r=$?; tail -3 $O/tests.log; [ $r -ne 0 ] && { grep -E "^E |FAIL" $O/tests.log | head -30; exit $r; }
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1
r=$?; tail -2 $O/smoke.log; [ $r -ne 0 ] && { tail -30 $O/smoke.log; exit $r; }
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
r=$?; tail -1 $O/bench.log | cut -c1-400; [ $r -ne 0 ] && { tail -30 $O/bench.log; exit $r; }
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $O/prof_7b -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > $O/prof_7b.log 2>&1
r=$?; echo "prof 7b rc=$r"; [ $r -ne 0 ] && { tail -20 $O/prof_7b.log; exit $r; }
python3 scripts/kernel_table.py $(find $O/prof_7b -name "*kernel_trace.csv" | head -1) > $O/kernels_7b.txt 2>&1; head -25 $O/kernels_7b.txt
rm -f $(find $O/prof_7b -name "*kernel_trace.csv") 2>/dev/null
exit 0
