#!/bin/bash
# Round 5 (z): ResNet50 b256 bf16 NHWC on the round-5 tree (auto conv routing), native-only conv, and the step's
# kernel table.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5z
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python -u scripts/bench_resnet50.py --steps 20 --warmup 5 > $O/rn50_auto.log 2>&1
r=$?; echo "auto: $(grep '^{' $O/rn50_auto.log | cut -c1-200)"; [ $r -ne 0 ] && { tail -30 $O/rn50_auto.log; exit $r; }
PADDLE2_AMD_CONV=native timeout -k 10 400 python -u scripts/bench_resnet50.py --steps 20 --warmup 5 > $O/rn50_native.log 2>&1
r=$?; echo "native: $(grep '^{' $O/rn50_native.log | cut -c1-200)"; [ $r -ne 0 ] && { tail -30 $O/rn50_native.log; exit $r; }
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/bench_resnet50.py --steps 5 --warmup 5 > $O/prof.log 2>&1
r=$?; echo "prof rc=$r"; [ $r -ne 0 ] && { tail -20 $O/prof.log; exit $r; }
python3 scripts/kernel_table.py $(find $O/prof -name "*kernel_trace.csv" | head -1) > $O/kernels.txt 2>&1; head -40 $O/kernels.txt
rm -f $(find $O/prof -name "*kernel_trace.csv") 2>/dev/null
exit 0
