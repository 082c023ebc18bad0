#!/bin/bash
# Round 6 (l3): ResNet50 with MIOpen Find: search + save the user find-db, then a second process seeded with it.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6l3
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
( while sleep 50; do date +%T >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 900 python -u scripts/bench_resnet50.py --steps 20 --warmup 5 --find-db "" --save-find-db $O/miopen_db \
  > $O/resnet_search.json 2> $O/resnet_search.err
r=$?; tail -1 $O/resnet_search.json | cut -c1-200; grep "warmup step 0" $O/resnet_search.err; [ $r -ne 0 ] && { kill $HB; tail -20 $O/resnet_search.err; exit $r; }
ls -la $O/miopen_db
timeout -k 10 600 python -u scripts/bench_resnet50.py --steps 20 --warmup 5 --find-db $O/miopen_db \
  > $O/resnet_seeded.json 2> $O/resnet_seeded.err
r=$?; kill $HB; tail -1 $O/resnet_seeded.json | cut -c1-200; grep "warmup step 0" $O/resnet_seeded.err; [ $r -ne 0 ] && { tail -20 $O/resnet_seeded.err; exit $r; }
exit 0
