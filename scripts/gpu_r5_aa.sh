#!/bin/bash
# Round 5 (aa): in-step A/B of existing knobs on the round-5 defaults (Llama-2-7B, 10 timed steps each): forward /
# dgrad tile-group heights (the gate|up forward now runs the plain forward GEMM), wgrad tile-group height, and the
# 8-wave causal flash forward.  Baseline first and last.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5aa
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
for v in "base:" "fwd8:PADDLE2_AMD_GEMM_GROUP_M_FWD=8" "fwd2:PADDLE2_AMD_GEMM_GROUP_M_FWD=2" \
         "dgrad8:PADDLE2_AMD_GEMM_GROUP_M_DGRAD=8" "wgrad4:PADDLE2_AMD_GEMM_GROUP_M_WGRAD=4" \
         "wgrad16:PADDLE2_AMD_GEMM_GROUP_M_WGRAD=16" "fa8:PADDLE2_AMD_FA_FWD_WAVES=8" "base2:"; do
  name=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/$name.log 2>&1
  r=$?; echo "$name: $(tail -1 $O/$name.log | cut -c1-150)"; [ $r -ne 0 ] && { tail -30 $O/$name.log; exit $r; }
done
exit 0
