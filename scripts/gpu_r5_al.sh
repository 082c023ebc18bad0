#!/bin/bash
# Round 5 (al): GPT-3 13B bf16 forward GEMM on W as stored (variant 6, no W^T transpose) vs the default TN v7.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5al
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
for v in default 6 default 6; do
  if [ $v = default ]; then unset PADDLE2_AMD_GEMM_VARIANT_FWD; else export PADDLE2_AMD_GEMM_VARIANT_FWD=$v; fi
  timeout -k 10 300 python -u bench.py --model gpt3-13b --seq-len 2048 --micro-batch 2 --steps 6 --warmup 3 > $O/b_$v.log 2>&1
  r=$?; echo "fwd=$v: $(tail -1 $O/b_$v.log | cut -c1-150)"; [ $r -ne 0 ] && { tail -30 $O/b_$v.log; exit $r; }
  echo "{\"fwd_variant\": \"$v\", \"bench\": $(tail -1 $O/b_$v.log)}" >> $O/fwd_variant.jsonl
done
exit 0
