#!/bin/bash
# Round 6 (c): kernel table of the split-dQ backward vs the fused atomic one.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6c
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/prof_flash_bwd_split.py 1 > $O/prof.log 2>&1
r=$?; [ $r -ne 0 ] && { tail -20 $O/prof.log; exit $r; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cat $f | cut -d, -f1-8 | head -20
rm -f $(find $O/prof -name "*kernel_trace.csv") 2>/dev/null
exit 0
