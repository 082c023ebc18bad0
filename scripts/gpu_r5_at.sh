#!/bin/bash
# Round 5 (at): few-row norm forward kernel — tests, then the decode step b1 / b16 with PADDLE2_AMD_NORM_ROW_MAXM=64
# (default) vs 0 (the one-wave-per-row kernel), and the Llama-2-7B bench (training rows take the old kernel).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5at
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_norm_rows_gpu.py tests/test_serving.py tests/test_main_grad_1d_gpu.py > $O/tests.log 2>&1
r=$?; tail -1 $O/tests.log; [ $r -ne 0 ] && { grep -E "^E |FAIL|Error" $O/tests.log | head -30; exit $r; }
for b in 1 16; do
  for m in 64 0 64; do
    PADDLE2_AMD_NORM_ROW_MAXM=$m timeout -k 10 240 python -u scripts/bench_serving.py --batch $b --prompt 1024 --new 64 > $O/b${b}_$m.log 2>&1
    r=$?; L=$(tail -1 $O/b${b}_$m.log); echo "b=$b row_maxm=$m: $(echo $L | grep -oE '"decode_ms_per_step": [0-9.]+')"; [ $r -ne 0 ] && { tail -20 $O/b${b}_$m.log; exit $r; }
    echo "{\"norm_row_maxm\": $m, \"run\": $L}" >> $O/norm_rows.jsonl
  done
done
exit 0
