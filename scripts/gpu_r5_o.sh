#!/bin/bash
# Round 5 (o): allocator / comm / new-feature GPU tests, the stage-3 collective path forced on one GPU at micro-batch
# 4 against the short-circuit (same memory class as an 8-GPU rank), then the measurements of script g.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5o
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_native_allocator.py tests/test_stage3_force_comm.py tests/test_native_pg_gpu.py tests/test_rccl_gpu.py \
  tests/test_fp8_gpu.py tests/test_decode_gemm_gpu.py "tests/test_gemm_gpu.py::test_tied_logits_native_matches_fp32" \
  > $O/tests.log 2>&1
r=$?; tail -2 $O/tests.log; [ $r -ne 0 ] && { grep -E "^E |FAIL" $O/tests.log | head -30; exit $r; }
for m in plain force; do
  f=0; [ $m = force ] && f=1
  PADDLE2_AMD_STAGE3_FORCE_COMM=$f timeout -k 10 300 python -u bench.py --micro-batch 4 --steps 8 --warmup 3 > $O/mb4_$m.log 2>&1
  r=$?; echo "mb4 $m: $(tail -1 $O/mb4_$m.log | cut -c1-160)"; [ $r -ne 0 ] && { tail -12 $O/mb4_$m.log; exit $r; }
done
bash scripts/gpu_r5_g.sh
