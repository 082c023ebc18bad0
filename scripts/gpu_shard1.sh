#!/bin/bash
# Sharding machinery overhead on one GPU: stage-3 wrapper (N==1 shortcuts, no collectives) vs plain step.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --shard-single --steps 4 --warmup 2 > gpurun_out/bench_shard1.log 2>&1
rc=$?; echo "shard-single rc=$rc"; tail -3 gpurun_out/bench_shard1.log
exit $rc
