#!/bin/bash
# ResNet50 DP bench on one MI355X (+ rocprofv3 kernel stats).
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/resnet
timeout -k 10 600 python -m pytest tests/test_batch_norm_gpu.py -x -q -m gpu > gpurun_out/resnet/bn_tests.log 2>&1 || { tail -30 gpurun_out/resnet/bn_tests.log; exit 1; }
tail -2 gpurun_out/resnet/bn_tests.log
timeout -k 10 600 python scripts/bench_resnet50.py --steps 20 --warmup 5 --batch 256 > gpurun_out/resnet/nhwc.json 2> gpurun_out/resnet/nhwc.err
cat gpurun_out/resnet/nhwc.json
timeout -k 10 600 python scripts/bench_resnet50.py --steps 20 --warmup 5 --batch 256 --data-format NCHW > gpurun_out/resnet/nchw.json 2> gpurun_out/resnet/nchw.err
cat gpurun_out/resnet/nchw.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/resnet/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/bench_resnet50.py" --steps 5 --warmup 3 --batch 256 > "$GRAFT_REPO_ROOT/gpurun_out/resnet/prof.log" 2>&1
cd "$GRAFT_REPO_ROOT"
f=$(find gpurun_out/resnet/prof -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY' > gpurun_out/resnet/top_kernels.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e6:.1f} ms")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:40]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {float(r["Percentage"]):6.2f}% n={r["Calls"]:>5} {r["Name"][:150]}')
PY
cat gpurun_out/resnet/top_kernels.txt | head -30
