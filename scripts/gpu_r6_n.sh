#!/bin/bash
# Round 6 (n): Llama-2-7B b64 decode — TunableOp selections for the hipBLASLt-routed wide projections.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6n
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
( while sleep 50; do date +%T >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 400 python -u scripts/bench_serving.py --batch 64 --gemm-autotune off > $O/base.json 2> $O/base.err
r=$?; tail -1 $O/base.json; [ $r -ne 0 ] && { kill $HB; tail -20 $O/base.err; exit $r; }
timeout -k 10 600 python -u scripts/bench_serving.py --batch 64 --new 8 --no-graph --gemm-autotune tune > $O/tune.json 2> $O/tune.err
r=$?; tail -1 $O/tune.json; [ $r -ne 0 ] && { kill $HB; tail -20 $O/tune.err; exit $r; }
cp tuning/gemm_gfx950.csv $O/gemm_gfx950.csv
timeout -k 10 400 python -u scripts/bench_serving.py --batch 64 --gemm-autotune auto > $O/tuned.json 2> $O/tuned.err
r=$?; kill $HB; tail -1 $O/tuned.json; [ $r -ne 0 ] && { tail -20 $O/tuned.err; exit $r; }
exit 0
