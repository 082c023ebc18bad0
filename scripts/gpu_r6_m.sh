#!/bin/bash
# Round 6 (m): GPT-3 13B fp8 step — hipBLASLt fp8 GEMM selections tuned by TunableOp (ScaledGemm) into the in-tree
# cache, then the step with the cache, against the step without it, on one box.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6m
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
( while sleep 50; do date +%T >> $O/heartbeat.txt; done ) &
HB=$!
A="--model gpt3-13b --fp8 --seq-len 2048 --micro-batch 2"
timeout -k 10 600 python -u bench.py $A --steps 5 --warmup 2 --gemm-autotune off > $O/base.log 2>&1
r=$?; tail -1 $O/base.log | cut -c1-260; [ $r -ne 0 ] && { kill $HB; tail -20 $O/base.log; exit $r; }
timeout -k 10 900 python -u bench.py $A --steps 2 --warmup 1 --gemm-autotune tune > $O/tune.log 2>&1
r=$?; tail -1 $O/tune.log | cut -c1-260; [ $r -ne 0 ] && { kill $HB; tail -20 $O/tune.log; exit $r; }
cp tuning/gemm_gfx950.csv $O/gemm_gfx950.csv
timeout -k 10 600 python -u bench.py $A --steps 5 --warmup 2 --gemm-autotune auto > $O/tuned.log 2>&1
r=$?; kill $HB; tail -1 $O/tuned.log | cut -c1-260; [ $r -ne 0 ] && { tail -20 $O/tuned.log; exit $r; }
wc -l $O/gemm_gfx950.csv
exit 0
