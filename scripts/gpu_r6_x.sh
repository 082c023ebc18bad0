#!/bin/bash
# Round 6 (x): tile-group height at the GPT-3 13B shapes (forward / wgrad / dgrad) and the Llama dgrad, then the
# Llama / GPT-3 13B steps with the wide-forward group rule.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6x
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
( while sleep 50; do date +%T >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 400 python -u scripts/exp_gemm_groupm_r6.py 4096 fwd_nn,wgrad,dgrad > $O/groupm_g13.jsonl 2> $O/groupm.err
r=$?; [ $r -ne 0 ] && { kill $HB; tail -20 $O/groupm.err; exit $r; }
timeout -k 10 400 python -u scripts/exp_gemm_groupm_r6.py 32768 dgrad > $O/groupm_dgrad.jsonl 2> $O/groupm2.err
r=$?; [ $r -ne 0 ] && { kill $HB; tail -20 $O/groupm2.err; exit $r; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_gemm_gpu.py \
  -k "fwd_nn or test_fwd" > $O/tests.log 2>&1
r=$?; tail -1 $O/tests.log; [ $r -ne 0 ] && { kill $HB; grep -E "^E |FAIL" $O/tests.log | head; exit $r; }
run() {  # name, env, args
  local n=$1; shift; local e=$1; shift
  env $e timeout -k 10 600 python -u bench.py "$@" > $O/$n.log 2>&1
  local r=$?; echo "$n $(tail -1 $O/$n.log | cut -c1-160)"; [ $r -ne 0 ] && { kill $HB; tail -20 $O/$n.log; exit $r; }
}
run llama_wide2 X=0 --steps 10 --warmup 3
run llama_wide4 PADDLE2_AMD_GEMM_GROUP_M_FWD_NN_WIDE=4 --steps 10 --warmup 3
kill $HB
exit 0
