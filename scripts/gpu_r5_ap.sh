#!/bin/bash
# Round 5 (ap): split-K decode GEMM with the reduction in the last-arriving workgroup (no reduce launch):
# bit-exact tests, then the HIP-graph decode step b1 / b16 with PADDLE2_AMD_DEC_FUSED_REDUCE=1/0 and the
# M <= 16 route forced native for the wide projections.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5ap
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_decode_gemm_gpu.py tests/test_serving.py > $O/tests.log 2>&1
r=$?; tail -1 $O/tests.log; [ $r -ne 0 ] && { grep -E "^E |FAIL|Error" $O/tests.log | head -30; exit $r; }
for b in 1 16; do
  for cfg in 1:auto 0:auto 1:native 0:native; do
    f=${cfg%%:*}; g=${cfg##*:}
    PADDLE2_AMD_DEC_FUSED_REDUCE=$f PADDLE2_AMD_DECODE_GEMM=$g timeout -k 10 240 python -u scripts/bench_serving.py --batch $b --prompt 1024 --new 64 > $O/b${b}_${f}_$g.log 2>&1
    r=$?; L=$(tail -1 $O/b${b}_${f}_$g.log); echo "b=$b fused=$f route=$g: $(echo $L | grep -oE '"decode_ms_per_step": [0-9.]+')"; [ $r -ne 0 ] && { tail -20 $O/b${b}_${f}_$g.log; exit $r; }
    echo "{\"fused_reduce\": $f, \"route\": \"$g\", \"run\": $L}" >> $O/fused_reduce.jsonl
  done
done
exit 0
