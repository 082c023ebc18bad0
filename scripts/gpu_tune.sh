#!/bin/bash
# Tune hipBLASLt GEMM selection for the flagship shapes (b=2 and b=4), then measure with the cache.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out tuning
export TMPDIR=/tmp
for b in 4 2; do
  PYTORCH_TUNABLEOP_VERBOSE=1 timeout -k 10 1500 python bench.py --steps 1 --warmup 1 --micro-batch $b --gemm-autotune tune > gpurun_out/tune_b$b.log 2>&1
  rc=$?; echo "tune b$b rc=$rc"; tail -2 gpurun_out/tune_b$b.log
  [ $rc -eq 0 ] || exit $rc
done
cp tuning/gemm_gfx950.csv gpurun_out/gemm_gfx950.csv
for b in 2 4; do
  timeout -k 10 900 python bench.py --steps 4 --warmup 2 --micro-batch $b > gpurun_out/bench_tuned_b$b.log 2>&1
  rc=$?; echo "bench tuned b$b rc=$rc"; tail -1 gpurun_out/bench_tuned_b$b.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 900 python bench.py --steps 4 --warmup 2 --micro-batch $b --gemm-autotune off > gpurun_out/bench_untuned_b$b.log 2>&1
  rc=$?; echo "bench untuned b$b rc=$rc"; tail -1 gpurun_out/bench_untuned_b$b.log
  [ $rc -eq 0 ] || exit $rc
done
