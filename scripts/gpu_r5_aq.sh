#!/bin/bash
# Round 5 (aq): M <= 16 decode GEMM route for the wide projections (qkv, gate|up: N > 8192) — native split-K vs
# hipBLASLt in the HIP-graph decode step at b = 1, 2, 4, 8.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5aq
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
for b in 1 2 4 8; do
  for g in auto native; do
    PADDLE2_AMD_DECODE_GEMM=$g timeout -k 10 240 python -u scripts/bench_serving.py --batch $b --prompt 1024 --new 64 > $O/b${b}_$g.log 2>&1
    r=$?; L=$(tail -1 $O/b${b}_$g.log); echo "b=$b route=$g: $(echo $L | grep -oE '"decode_ms_per_step": [0-9.]+')"; [ $r -ne 0 ] && { tail -20 $O/b${b}_$g.log; exit $r; }
    echo "{\"route\": \"$g\", \"run\": $L}" >> $O/route.jsonl
  done
done
exit 0
