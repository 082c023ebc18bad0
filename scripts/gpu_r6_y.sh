#!/bin/bash
# Round 6 (y): kernel statistics of the Llama-2-7B serving decode at b1 and b64 (HIP-graph decode, 64 new tokens).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6y
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
for b in 1 64; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_b$b -o run --output-format csv -- python3 scripts/bench_serving.py --batch $b > $O/serve_b$b.log 2>&1
  r=$?; echo "b$b rc=$r $(grep decode_ms $O/serve_b$b.log | tail -1 | cut -c1-300)"; [ $r -ne 0 ] && { tail -20 $O/serve_b$b.log; exit $r; }
  f=$(find $O/prof_b$b -name "*kernel_stats.csv" | head -1); head -30 $f | cut -d, -f1-5 > $O/stats_b$b.txt
  rm -f $(find $O/prof_b$b -name "*kernel_trace.csv") 2>/dev/null
done
exit 0
