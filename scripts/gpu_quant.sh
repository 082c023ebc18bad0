#!/bin/bash
# Weight-only kernel numerics + decode-shape timing on one MI355X.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/quant
timeout -k 10 600 python -m pytest tests/test_quantization.py -x -q -m gpu > gpurun_out/quant/tests.log 2>&1 || { tail -40 gpurun_out/quant/tests.log; exit 1; }
tail -2 gpurun_out/quant/tests.log
timeout -k 10 300 python scripts/bench_weight_only.py > gpurun_out/quant/bench.jsonl 2> gpurun_out/quant/bench.err
cat gpurun_out/quant/bench.jsonl
