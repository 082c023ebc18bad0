#!/bin/bash
# Round 5 (ak): GPT-3 13B fp8 and bf16 step kernel tables at HEAD (bias / norm-weight gradients into the fp32
# main-grad slots, deferred fp8 scale updates).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5ak
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
for m in fp8 bf16; do
  F=""; [ $m = fp8 ] && F="--fp8"
  timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $O/prof_$m -o run --output-format csv -- python3 bench.py --model gpt3-13b $F --seq-len 2048 --micro-batch 2 --steps 3 --warmup 2 > $O/prof_$m.log 2>&1
  r=$?; echo "prof $m rc=$r: $(tail -1 $O/prof_$m.log | cut -c1-140)"; [ $r -ne 0 ] && { tail -20 $O/prof_$m.log; exit $r; }
  python3 scripts/kernel_table.py $(find $O/prof_$m -name "*kernel_trace.csv" | head -1) > $O/kernels_$m.txt 2>&1; head -40 $O/kernels_$m.txt
  rm -f $(find $O/prof_$m -name "*kernel_trace.csv") 2>/dev/null
done
exit 0
