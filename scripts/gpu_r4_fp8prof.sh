#!/bin/bash
# Round 4: GPT-3 13B fp8 step kernel table (auto fp8 GEMM routes).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4fp8prof
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --model gpt3-13b --fp8 --seq-len 2048 --micro-batch 2 --steps 3 --warmup 2 > $O/prof.log 2>&1
r=$?; echo "prof rc=$r"; [ $r -ne 0 ] && { tail -20 $O/prof.log; exit $r; }
python3 scripts/kernel_table.py $(find $O/prof -name "*kernel_trace.csv" | head -1) > $O/kernels.txt 2>&1; head -25 $O/kernels.txt
exit 0
