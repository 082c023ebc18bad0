#!/bin/bash
# Round 4: K-rotation of odd slots (store-burst staggering) and non-temporal epilogue stores on the spread kernel.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4rot
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python3 -u scripts/bench_gemm_v7.py 448,960,1472,1984 > $O/bench.jsonl 2> $O/bench.err
echo "bench rc=$?"
