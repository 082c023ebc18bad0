#!/bin/bash
# Round 6 (ag): split-K workgroup target of the M <= 16 decode GEMM (PADDLE2_AMD_DEC_WG_TARGET; default 1024) at
# decode b1 / b16.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6ag
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
( while sleep 50; do date +%T >> $O/heartbeat.txt; done ) &
HB=$!
for b in 1 16; do
  for t in 1024 512 2048 768; do
    PADDLE2_AMD_DEC_WG_TARGET=$t timeout -k 10 400 python -u scripts/bench_serving.py --batch $b > $O/serve_b${b}_t$t.json 2> $O/serve_b${b}_t$t.err
    r=$?; echo "b$b target=$t $(grep -o '"decode_ms_per_step": [0-9.]*' $O/serve_b${b}_t$t.json)"; [ $r -ne 0 ] && { kill $HB; tail -20 $O/serve_b${b}_t$t.err; exit $r; }
  done
done
kill $HB
exit 0
