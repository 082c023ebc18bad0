#!/bin/bash
# Round 4 close-out: the flagship bench at the committed defaults (N=1) and its rocprofv3 kernel table.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4close
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 420 python3 -u bench.py --steps 10 --warmup 3 > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '"metric"' $O/bench.log | cut -c1-300; [ $rc -ne 0 ] && { tail -30 $O/bench.log; exit $rc; }
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > $O/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/prof.log; exit $rc; }
python3 scripts/kernel_table.py $(find $O/prof -name "*kernel_trace.csv" | head -1) > $O/kernels.txt 2>&1; head -30 $O/kernels.txt
exit 0
