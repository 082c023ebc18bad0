#!/bin/bash
# Round 4: the GPU test tier + smoke, then the secondary configs with the per-shape routes (bf16 GEMM routing
# measured for GPT, fp8 GEMM auto, conv auto) — compare with gpurun_out/r4sec (static routes).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4routes
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
bash scripts/gpu_r4_fulltests.sh; rc=$?
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 600 python3 -u bench.py --model gpt3-13b --seq-len 2048 --micro-batch 2 --steps 5 --warmup 2 > $O/gpt13b_bf16.log 2>&1
r=$?; echo "gpt13b bf16 rc=$r"; grep -h '"metric"' $O/gpt13b_bf16.log | cut -c1-200; [ $r -ne 0 ] && { tail -20 $O/gpt13b_bf16.log; exit $r; }
timeout -k 10 600 python3 -u bench.py --model gpt3-13b --fp8 --seq-len 2048 --micro-batch 2 --steps 5 --warmup 2 > $O/gpt13b_fp8.log 2>&1
r=$?; echo "gpt13b fp8 rc=$r"; grep -h '"metric"' $O/gpt13b_fp8.log | cut -c1-200; [ $r -ne 0 ] && { tail -20 $O/gpt13b_fp8.log; exit $r; }
timeout -k 10 400 python3 -u scripts/bench_resnet50.py --steps 20 --warmup 5 --batch 256 > $O/resnet_auto.json 2> $O/resnet_auto.err
r=$?; echo "resnet auto rc=$r"; cat $O/resnet_auto.json; [ $r -ne 0 ] && { tail -20 $O/resnet_auto.err; exit $r; }
exit $rc
