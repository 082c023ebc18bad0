#!/bin/bash
# rocprofv3 kernel-trace profile of the default bench config (Llama-2-7B b=8 s=4096), 1 warmup + 2 timed steps.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8 -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 > gpurun_out/bench_prof8.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/bench_prof8.log
[ $rc -eq 0 ] || exit $rc
python3 - <<'PY' > gpurun_out/top_kernels_b8.txt
import csv
rows = list(csv.DictReader(open("gpurun_out/prof8/run_kernel_stats.csv")))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total kernel time {tot/1e6:.1f} ms over 3 steps (incl. init)")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:45]:
    print(f"{float(r['TotalDurationNs'])/3e6:8.2f} ms/step {int(r['Calls'])/3:7.1f} calls {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:110]}")
PY
cat gpurun_out/top_kernels_b8.txt
