#!/bin/bash
# Round 6 (g): fast-reciprocal sigmoid/SiLU in the GEMM epilogues and elementwise kernels — numerics of every
# activation path, then an in-step A/B of the SwiGLU routes (unfused default, fused forward epilogue, one-node MLP).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6g
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gemm_gpu.py tests/test_fused_act.py tests/test_decode_gemm_gpu.py tests/test_kernels_gpu.py > $O/tests.log 2>&1
r=$?; tail -3 $O/tests.log; [ $r -ne 0 ] && { grep -E "^E |FAIL" $O/tests.log | head -30; exit $r; }
for v in default fwd_fused mlp_node both; do
  case $v in
    default) E="" ;;
    fwd_fused) E="PADDLE2_AMD_SWIGLU_FWD=fused" ;;
    mlp_node) E="PADDLE2_AMD_SWIGLU_MLP_NODE=1" ;;
    both) E="PADDLE2_AMD_SWIGLU_FWD=fused PADDLE2_AMD_SWIGLU_MLP_NODE=1" ;;
  esac
  env $E timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > $O/bench_$v.log 2>&1
  r=$?; echo "$v: $(tail -1 $O/bench_$v.log | grep -o '"ms_per_step": [0-9.]*')"; [ $r -ne 0 ] && { tail -20 $O/bench_$v.log; exit $r; }
done
exit 0
