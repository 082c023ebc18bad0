#!/bin/bash
# Round 5 (af): the forward GEMM on W as stored (v6, B not K-major: no per-step W^T transpose) vs the TN v7
# forward on W^T — GPT-3 13B bf16 (short K, 161 transposes per step) and Llama-2-7B, plus forward-GEMM numerics.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5af
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
PADDLE2_AMD_GEMM_VARIANT_FWD=6 timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  -p no:cacheprovider -m gpu tests/test_gemm_gpu.py tests/test_llama_gpu.py > $O/tests.log 2>&1
r=$?; tail -2 $O/tests.log; [ $r -ne 0 ] && { grep -E "^E |FAIL" $O/tests.log | head -30; exit $r; }
for v in "gpt_base:--model gpt3-13b --seq-len 2048 --micro-batch 2:" "gpt_v6:--model gpt3-13b --seq-len 2048 --micro-batch 2:PADDLE2_AMD_GEMM_VARIANT_FWD=6" \
         "llama_base::" "llama_v6::PADDLE2_AMD_GEMM_VARIANT_FWD=6" "gpt_base2:--model gpt3-13b --seq-len 2048 --micro-batch 2:"; do
  name=${v%%:*}; rest=${v#*:}; a=${rest%%:*}; envs=${rest#*:}
  env $envs timeout -k 10 300 python -u bench.py $a --steps 8 --warmup 3 > $O/$name.log 2>&1
  r=$?; echo "$name: $(tail -1 $O/$name.log | cut -c1-150)"; [ $r -ne 0 ] && { tail -30 $O/$name.log; exit $r; }
done
exit 0
