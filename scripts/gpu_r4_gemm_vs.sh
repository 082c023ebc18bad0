#!/bin/bash
# Round 4: the spread three-barrier schedule (v7 SCHED bit 7: variants 192 / 194 / 258) vs v6 / v9 / hipBLASLt.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4vs
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python3 -u scripts/bench_gemm_v7.py 9,192,194,258 > $O/bench.jsonl 2> $O/bench.err
echo "bench rc=$?"
