#!/bin/bash
# Round 4: spread schedule + 16-B epilogue stores (variant 448 = v7 SCHED 384) and the grouped tile order sweep.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4x4
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python3 -u scripts/bench_gemm_v7.py 192,448 > $O/bench_g8.jsonl 2> $O/bench_g8.err || exit $?
for g in 4 16; do
  PADDLE2_AMD_GEMM_GROUP_M=$g timeout -k 10 300 python3 -u scripts/bench_gemm_v7.py 448 > $O/bench_g$g.jsonl 2> $O/bench_g$g.err || exit $?
done
echo done
