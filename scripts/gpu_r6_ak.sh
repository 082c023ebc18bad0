#!/bin/bash
# Round 6 (ak): b1 decode kernel statistics with the 768 split-K workgroup target (rocprofv3 kernel trace + stats).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6ak
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o b1 --output-format csv -- python3 -u scripts/bench_serving.py --batch 1 > $O/b1.log 2>&1
r=$?; tail -2 $O/b1.log; [ $r -ne 0 ] && exit $r
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/decode_b1_kernel_stats.csv \;
head -12 $O/decode_b1_kernel_stats.csv | cut -c1-200
