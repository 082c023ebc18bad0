#!/bin/bash
# Round 6 (ai): decode split-K target 768 as the default: decode / serving GPU tests and the serving bench at b1 / b16 / b64.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6ai
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_decode_gemm_gpu.py tests/test_serving.py tests/test_quantization.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for b in 1 16 64; do
  timeout -k 10 400 python -u scripts/bench_serving.py --batch $b > $O/serve_b$b.json 2> $O/serve_b$b.err || { tail -20 $O/serve_b$b.err; exit 1; }
  echo "b$b $(grep -o '"decode_ms_per_step": [0-9.]*' $O/serve_b$b.json)"
done
