#!/bin/bash
# Round 6 (aj): the 768 split target at b4 / b8 (vs 1024), and b16 with every projection on the split-K kernel
# (PADDLE2_AMD_DECODE_GEMM=native) vs auto (wide qkv / gate|up on hipBLASLt), interleaved x2.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6aj
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
run() {  # tag, batch, env...
  local tag=$1 b=$2; shift 2
  env "$@" timeout -k 10 400 python -u scripts/bench_serving.py --batch $b > $O/$tag.json 2> $O/$tag.err
  local r=$?; echo "$tag $(grep -o '"decode_ms_per_step": [0-9.]*' $O/$tag.json)"; return $r
}
for rep in 1 2; do
  for b in 4 8; do
    run b${b}_t768_r$rep $b PADDLE2_AMD_DEC_WG_TARGET=768 || exit 1
    run b${b}_t1024_r$rep $b PADDLE2_AMD_DEC_WG_TARGET=1024 || exit 1
  done
  run b16_auto_r$rep 16 PADDLE2_AMD_DECODE_GEMM=auto || exit 1
  run b16_native_r$rep 16 PADDLE2_AMD_DECODE_GEMM=native || exit 1
done
