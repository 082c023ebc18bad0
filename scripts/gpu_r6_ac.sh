#!/bin/bash
# Round 6 (ac): secondary ResNet50 b256 number at HEAD (seeded MIOpen find-db, auto conv routing) and an interleaved
# Llama A/B of the forward on W as stored (default) vs the TN forward on W^T (PADDLE2_AMD_GEMM_FWD_NN_MAX_M=0).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6ac
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
( while sleep 50; do date +%T >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 600 python -u scripts/bench_resnet50.py --steps 20 --warmup 5 > $O/resnet.json 2> $O/resnet.err
r=$?; tail -1 $O/resnet.json | cut -c1-200; [ $r -ne 0 ] && { kill $HB; tail -20 $O/resnet.err; exit $r; }
run() {  # name, env, args
  local n=$1; shift; local e=$1; shift
  env $e timeout -k 10 600 python -u bench.py "$@" > $O/$n.log 2>&1
  local r=$?; echo "$n $(grep -o '"value": [0-9.]*' $O/$n.log | tail -1)"; [ $r -ne 0 ] && { kill $HB; tail -20 $O/$n.log; exit $r; }
}
run nn_a X=0 --steps 10 --warmup 3
run tn_a PADDLE2_AMD_GEMM_FWD_NN_MAX_M=0 --steps 10 --warmup 3
run nn_b X=0 --steps 10 --warmup 3
run tn_b PADDLE2_AMD_GEMM_FWD_NN_MAX_M=0 --steps 10 --warmup 3
kill $HB
exit 0
