#!/bin/bash
# Round 4 secondary configs: GPT-3 13B bf16 (fused GELU MLP on / off), GPT-3 13B fp8 (native fp8 GEMM vs hipBLASLt),
# ResNet-50 (native 1x1 / 3x3 convs vs MIOpen).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4sec
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
bash scripts/gpu_r4_fulltests.sh || exit $?
for f in 1 0; do
  PADDLE2_AMD_FUSED_GELU_MLP=$f timeout -k 10 600 python3 -u bench.py --model gpt3-13b --seq-len 2048 --micro-batch 2 --steps 5 --warmup 2 > $O/gpt13b_fused$f.log 2>&1
  rc=$?; echo "gpt13b fused=$f rc=$rc"; grep '"metric"' $O/gpt13b_fused$f.log | cut -c1-200; [ $rc -ne 0 ] && { tail -20 $O/gpt13b_fused$f.log; exit $rc; }
done
for g in native blas; do
  PADDLE2_AMD_FP8_GEMM=$g timeout -k 10 600 python3 -u bench.py --model gpt3-13b --fp8 --seq-len 2048 --micro-batch 2 --steps 5 --warmup 2 > $O/gpt13b_fp8_$g.log 2>&1
  rc=$?; echo "gpt13b fp8 $g rc=$rc"; grep '"metric"' $O/gpt13b_fp8_$g.log | cut -c1-200; [ $rc -ne 0 ] && { tail -20 $O/gpt13b_fp8_$g.log; exit $rc; }
done
for c in native miopen; do
  PADDLE2_AMD_CONV=$c timeout -k 10 400 python3 -u scripts/bench_resnet50.py --steps 20 --warmup 5 --batch 256 > $O/resnet_$c.json 2> $O/resnet_$c.err
  rc=$?; echo "resnet $c rc=$rc"; cat $O/resnet_$c.json; [ $rc -ne 0 ] && { tail -20 $O/resnet_$c.err; exit $rc; }
done
exit 0
