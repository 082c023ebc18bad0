#!/bin/bash
# Round 5 (ae): GPT-3 13B bf16 (b2 s2048) wgrad tile-group height A/B (short-K, fp32-epilogue weight gradients).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5ae
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
for v in "base:" "wg4:PADDLE2_AMD_GEMM_GROUP_M_WGRAD=4" "wg16:PADDLE2_AMD_GEMM_GROUP_M_WGRAD=16" "wg2:PADDLE2_AMD_GEMM_GROUP_M_WGRAD=2" "base2:"; do
  name=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 300 python -u bench.py --model gpt3-13b --seq-len 2048 --micro-batch 2 --steps 8 --warmup 3 > $O/$name.log 2>&1
  r=$?; echo "$name: $(tail -1 $O/$name.log | cut -c1-150)"; [ $r -ne 0 ] && { tail -30 $O/$name.log; exit $r; }
done
exit 0
