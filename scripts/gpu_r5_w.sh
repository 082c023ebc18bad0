#!/bin/bash
# Round 5 (w): stage 3 keeping units gathered from forward to backward (no backward all-gathers) on the GPU comm
# path — force-comm numerics, then the 7B forced-comm step at micro-batch 4 with and without it.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5w
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_stage3_force_comm.py > $O/tests.log 2>&1
r=$?; tail -2 $O/tests.log; [ $r -ne 0 ] && { grep -E "^E |FAIL" $O/tests.log | head -30; exit $r; }
for k in 0 1; do
  PADDLE2_AMD_BENCH_DEBUG=1 PADDLE2_AMD_STAGE3_FORCE_COMM=1 PADDLE2_AMD_STAGE3_KEEP_GATHERED=$k timeout -k 10 400 \
    python -u bench.py --micro-batch 4 --steps 8 --warmup 3 > $O/force_mb4_keep$k.log 2>&1
  r=$?; echo "keep $k: $(grep '^\[bench\] warmup step 2' $O/force_mb4_keep$k.log | cut -c1-160) $(tail -1 $O/force_mb4_keep$k.log | cut -c1-160)"
  [ $r -ne 0 ] && { tail -30 $O/force_mb4_keep$k.log; exit $r; }
done
exit 0
