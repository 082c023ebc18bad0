#!/bin/bash
# Round 6 (l): ResNet50 b256 bf16 NHWC: MIOpen Find (FLAGS_cudnn_exhaustive_search) on / off, auto conv routing.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6l
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
for ex in 0 1; do
  timeout -k 10 600 python -u scripts/bench_resnet50.py --steps 20 --warmup 5 --exhaustive-search $ex \
    > $O/resnet_ex$ex.json 2> $O/resnet_ex$ex.err
  r=$?; tail -1 $O/resnet_ex$ex.json | cut -c1-300; [ $r -ne 0 ] && { tail -20 $O/resnet_ex$ex.err; exit $r; }
done
exit 0
