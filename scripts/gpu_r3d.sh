#!/bin/bash
# bias-grad kernel test, GPT-3 13B (b2 s2048, accumulate 1 and 4), Llama-2-7B headline bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r3d
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
    tests/test_native_allocator.py > gpurun_out/r3d/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r3d/tests.log; [ $rc -eq 0 ] || exit $rc
for acc in 1 4; do
  timeout -k 10 500 python -u bench.py --model gpt3-13b --seq-len 2048 --micro-batch 2 --accumulate-steps $acc \
      --steps 3 --warmup 1 > gpurun_out/r3d/gpt_acc$acc.log 2>&1
  rc=$?; echo "gpt acc=$acc rc=$rc"; grep '"metric"' gpurun_out/r3d/gpt_acc$acc.log | cut -c1-420; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/r3d/bench.log 2>&1
rc=$?; grep '"metric"' gpurun_out/r3d/bench.log | cut -c1-300; exit $rc
