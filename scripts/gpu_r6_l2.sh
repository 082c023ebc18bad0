#!/bin/bash
# Round 6 (l2): ResNet50 with MIOpen Find — how long the search takes on a fresh box and what it buys.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6l2
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
( while sleep 50; do date +%T >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 1000 python -u scripts/bench_resnet50.py --steps 20 --warmup 5 --exhaustive-search 1 \
  > $O/resnet_ex1.json 2> $O/resnet_ex1.err
r=$?; kill $HB; tail -1 $O/resnet_ex1.json | cut -c1-300; grep warmup $O/resnet_ex1.err; [ $r -ne 0 ] && { tail -20 $O/resnet_ex1.err; exit $r; }
exit 0
