#!/bin/bash
# Round 4 close-out: the GPU test tier + smoke, then the GPT-3 13B bf16 and ResNet50 kernel tables (rocprofv3).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4final
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
bash scripts/gpu_r4_fulltests.sh; rc=$?
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $O/prof_gpt -o run --output-format csv -- python3 bench.py --model gpt3-13b --seq-len 2048 --micro-batch 2 --steps 3 --warmup 2 > $O/prof_gpt.log 2>&1
r=$?; echo "prof gpt rc=$r"; [ $r -ne 0 ] && { tail -20 $O/prof_gpt.log; exit $r; }
python3 scripts/kernel_table.py $(find $O/prof_gpt -name "*kernel_trace.csv" | head -1) > $O/kernels_gpt.txt 2>&1; head -30 $O/kernels_gpt.txt
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $O/prof_resnet -o run --output-format csv -- python3 scripts/bench_resnet50.py --steps 10 --warmup 5 --batch 256 > $O/prof_resnet.log 2>&1
r=$?; echo "prof resnet rc=$r"; [ $r -ne 0 ] && { tail -20 $O/prof_resnet.log; exit $r; }
python3 scripts/kernel_table.py $(find $O/prof_resnet -name "*kernel_trace.csv" | head -1) > $O/kernels_resnet.txt 2>&1; head -30 $O/kernels_resnet.txt
exit $rc
