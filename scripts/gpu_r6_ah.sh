#!/bin/bash
# Round 6 (ah): decode split-K workgroup target 768 vs 1024 (default), interleaved repeats at b1 / b16, plus 640 / 896.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6ah
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
( while sleep 50; do date +%T >> $O/heartbeat.txt; done ) &
HB=$!
for rep in 1 2; do
for b in 1 16; do
  for t in 1024 768 640 896; do
    PADDLE2_AMD_DEC_WG_TARGET=$t timeout -k 10 400 python -u scripts/bench_serving.py --batch $b > $O/serve_b${b}_t${t}_r$rep.json 2> $O/serve_b${b}_t${t}_r$rep.err
    r=$?; echo "rep$rep b$b target=$t $(grep -o '"decode_ms_per_step": [0-9.]*' $O/serve_b${b}_t${t}_r$rep.json)"; [ $r -ne 0 ] && { kill $HB; tail -20 $O/serve_b${b}_t${t}_r$rep.err; exit $r; }
  done
done
done
kill $HB
exit 0
