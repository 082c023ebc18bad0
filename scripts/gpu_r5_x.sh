#!/bin/bash
# Round 5 (x): GPT-3 13B bf16 (b2 s2048) on the round-5 defaults: step time and its kernel table.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5x
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python -u bench.py --model gpt3-13b --seq-len 2048 --micro-batch 2 --steps 8 --warmup 3 > $O/bf16_13b.log 2>&1
r=$?; echo "bf16 13b: $(tail -1 $O/bf16_13b.log | cut -c1-220)"; [ $r -ne 0 ] && { tail -30 $O/bf16_13b.log; exit $r; }
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --model gpt3-13b --seq-len 2048 --micro-batch 2 --steps 3 --warmup 2 > $O/prof.log 2>&1
r=$?; echo "prof rc=$r"; [ $r -ne 0 ] && { tail -20 $O/prof.log; exit $r; }
python3 scripts/kernel_table.py $(find $O/prof -name "*kernel_trace.csv" | head -1) > $O/kernels.txt 2>&1; head -32 $O/kernels.txt
rm -f $(find $O/prof -name "*kernel_trace.csv") 2>/dev/null
exit 0
