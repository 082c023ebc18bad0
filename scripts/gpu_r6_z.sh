#!/bin/bash
# Round 6 (z): decode split-K partials handed to the residual-add + RMSNorm (no reduce launch) — serving GPU tests,
# then the decode bench at b1 / b16 / b64 with and without the handoff.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6z
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
( while sleep 50; do date +%T >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_serving.py tests/test_decode_gemm_gpu.py tests/test_norm_rows_gpu.py > $O/tests.log 2>&1
r=$?; tail -2 $O/tests.log; [ $r -ne 0 ] && { kill $HB; grep -E "^E |FAIL|Error" $O/tests.log | head -30; exit $r; }
for b in 1 16 64; do
  for on in 1 0; do
    PADDLE2_AMD_DEC_PARTIALS=$on timeout -k 10 400 python -u scripts/bench_serving.py --batch $b > $O/serve_b${b}_p$on.json 2> $O/serve_b${b}_p$on.err
    r=$?; echo "b$b partials=$on $(grep -o '"decode_ms_per_step": [0-9.]*' $O/serve_b${b}_p$on.json)"; [ $r -ne 0 ] && { kill $HB; tail -20 $O/serve_b${b}_p$on.err; exit $r; }
  done
done
kill $HB
exit 0
