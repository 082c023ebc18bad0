#!/bin/bash
# Round 5 (av): split-K reduce with its partial loads unrolled — decode tests and the decode step b1 / b16.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5av
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_decode_gemm_gpu.py tests/test_serving.py tests/test_quantization.py > $O/tests.log 2>&1
r=$?; tail -1 $O/tests.log; [ $r -ne 0 ] && { grep -E "^E |FAIL|Error" $O/tests.log | head -30; exit $r; }
for b in 1 16 1 16; do
  timeout -k 10 240 python -u scripts/bench_serving.py --batch $b --prompt 1024 --new 64 > $O/b$b.log 2>&1
  r=$?; L=$(tail -1 $O/b$b.log); echo "b=$b: $(echo $L | grep -oE '"decode_ms_per_step": [0-9.]+')"; [ $r -ne 0 ] && { tail -20 $O/b$b.log; exit $r; }
  echo "$L" >> $O/serving.jsonl
done
exit 0
