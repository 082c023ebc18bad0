#!/bin/bash
# Round 5 (ao): decode-attention KV split sizing (PADDLE2_AMD_DECODE_WG_TARGET / _SPLIT_TOKENS) on the HIP-graph
# decode step, b1 / b16 / b64, Llama-2-7B, prompt 1024 + 64 new tokens.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5ao
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_serving.py > $O/tests.log 2>&1
r=$?; tail -1 $O/tests.log; [ $r -ne 0 ] && { grep -E "^E |FAIL" $O/tests.log | head -30; exit $r; }
for b in 1 16 64; do
  for cfg in 2048:64 4096:64 4096:32 2048:32 8192:32; do
    t=${cfg%%:*}; k=${cfg##*:}
    PADDLE2_AMD_DECODE_WG_TARGET=$t PADDLE2_AMD_DECODE_SPLIT_TOKENS=$k timeout -k 10 240 python -u scripts/bench_serving.py --batch $b --prompt 1024 --new 64 > $O/b${b}_$t_$k.log 2>&1
    r=$?; L=$(tail -1 $O/b${b}_$t_$k.log); echo "b=$b target=$t tok=$k: $(echo $L | cut -c1-260)"; [ $r -ne 0 ] && { tail -20 $O/b${b}_$t_$k.log; exit $r; }
    echo "{\"wg_target\": $t, \"split_tokens\": $k, \"run\": $L}" >> $O/split_sweep.jsonl
  done
done
exit 0
