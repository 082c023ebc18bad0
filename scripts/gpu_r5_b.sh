#!/bin/bash
# Round 5 (b): flash bwd 4- vs 8-wave A/B, GEMM epilogue study, the new GPU tests, forced-comm vs plain 7B bench.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5b
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python -u scripts/exp_flash_bwd_waves.py 3 > $O/fa_bwd_waves.jsonl 2> $O/fa_bwd_waves.err
r=$?; cat $O/fa_bwd_waves.jsonl; [ $r -ne 0 ] && { tail -20 $O/fa_bwd_waves.err; exit $r; }
timeout -k 10 400 python -u scripts/exp_gemm_epi.py 3 > $O/gemm_epi.jsonl 2> $O/gemm_epi.err
r=$?; cat $O/gemm_epi.jsonl; [ $r -ne 0 ] && { tail -20 $O/gemm_epi.err; exit $r; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_stage3_force_comm.py tests/test_ipc_allreduce.py tests/test_fused_act.py tests/test_comm_context_gpu.py \
  tests/test_native_pg_gpu.py tests/test_bench_configs.py > $O/tests.log 2>&1
r=$?; tail -3 $O/tests.log; [ $r -ne 0 ] && { grep -E "^E |FAIL" $O/tests.log | head -30; exit $r; }
PADDLE2_AMD_STAGE3_FORCE_COMM=1 timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > $O/bench_force.log 2>&1
r=$?; tail -1 $O/bench_force.log; [ $r -ne 0 ] && { tail -30 $O/bench_force.log; exit $r; }
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > $O/bench_plain.log 2>&1
r=$?; tail -1 $O/bench_plain.log; [ $r -ne 0 ] && { tail -30 $O/bench_plain.log; exit $r; }
exit 0
