#!/bin/bash
# Round 4: per-shape route timing with more iterations (fp8 GEMM 10, conv fwd+bwd 5): GPT-3 13B fp8, ResNet50.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4routes2
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 python3 -u bench.py --model gpt3-13b --fp8 --seq-len 2048 --micro-batch 2 --steps 5 --warmup 2 > $O/gpt13b_fp8.log 2>&1
r=$?; echo "gpt13b fp8 rc=$r"; grep -h '"metric"' $O/gpt13b_fp8.log | cut -c1-200; [ $r -ne 0 ] && { tail -20 $O/gpt13b_fp8.log; exit $r; }
timeout -k 10 400 python3 -u scripts/bench_resnet50.py --steps 20 --warmup 5 --batch 256 > $O/resnet_auto.json 2> $O/resnet_auto.err
r=$?; echo "resnet auto rc=$r"; cat $O/resnet_auto.json; grep "conv routes" $O/resnet_auto.err | head -40; [ $r -ne 0 ] && { tail -20 $O/resnet_auto.err; exit $r; }
exit 0
