#!/bin/bash
# Round 5 (d): forced-comm test (noise-aware), flash fwd / bwd timing after the restructure, 7B bench plain + forced.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5d
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python -u scripts/bench_flash_fwd.py > $O/fa_fwd.jsonl 2> $O/fa_fwd.err
r=$?; cat $O/fa_fwd.jsonl; [ $r -ne 0 ] && { tail -20 $O/fa_fwd.err; exit $r; }
timeout -k 10 300 python -u scripts/exp_flash_bwd_waves.py 2 > $O/fa_bwd.jsonl 2> $O/fa_bwd.err
r=$?; cat $O/fa_bwd.jsonl; [ $r -ne 0 ] && { tail -20 $O/fa_bwd.err; exit $r; }
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > $O/bench_plain.log 2>&1
r=$?; tail -1 $O/bench_plain.log; [ $r -ne 0 ] && { tail -30 $O/bench_plain.log; exit $r; }
PADDLE2_AMD_STAGE3_FORCE_COMM=1 timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > $O/bench_force.log 2>&1
r=$?; tail -1 $O/bench_force.log; [ $r -ne 0 ] && { tail -30 $O/bench_force.log; exit $r; }
timeout -k 10 300 python -u scripts/exp_decode64.py > $O/dec64.jsonl 2> $O/dec64.err
r=$?; cat $O/dec64.jsonl; [ $r -ne 0 ] && { tail -20 $O/dec64.err; exit $r; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_decode_gemm_gpu.py tests/test_stage3_force_comm.py tests/test_ipc_allreduce.py tests/test_fused_act.py tests/test_comm_context_gpu.py \
  tests/test_native_pg_gpu.py tests/test_bench_configs.py > $O/tests.log 2>&1
r=$?; tail -3 $O/tests.log; [ $r -ne 0 ] && { grep -E "^E |FAIL" $O/tests.log | head -30; exit $r; }
exit 0
